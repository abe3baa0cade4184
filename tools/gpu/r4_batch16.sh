#!/bin/bash
# Stream-priority A/Bs of batch14 + batch15 (closing span table) in one box.
set -o pipefail
bash tools/gpu/r4_batch14.sh && bash tools/gpu/r4_batch15.sh
