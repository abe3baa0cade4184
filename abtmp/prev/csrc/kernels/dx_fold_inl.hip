// Two-phase range-verification Miller fold with every tower / curve function
// force-inlined into the kernels (one register allocation per kernel, no
// call frames).  Body: fold_body.h.
#define DX_NI __host__ __device__ __forceinline__
#define FOLD_SFX inl
#include "fold_body.h"
