// Two-phase range-verification Miller fold, tower functions out of line
// (small code, call frames).  Body: fold_body.h.
#define FOLD_SFX ni
#include "fold_body.h"
