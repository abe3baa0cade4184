#!/bin/bash
# Which engine does a 512 MB device-to-host copy (ledger payloads): kernel +
# memory-copy trace of tools/d2h_probe.py, default env and SDMA forced on.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/d2h -o run -- python3 -u tools/d2h_probe.py > gpurun_out/d2h.log 2>&1 || { tail -20 gpurun_out/d2h.log; exit 1; }
grep -E "ms|GB" gpurun_out/d2h.log | grep -v rocprof
python3 - <<'PY'
import csv, glob, collections
k = glob.glob("gpurun_out/d2h/**/*kernel_trace.csv", recursive=True)
m = glob.glob("gpurun_out/d2h/**/*memory_copy_trace.csv", recursive=True)
c = collections.Counter()
for r in csv.DictReader(open(k[0])):
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    if d > 1:
        c[r["Kernel_Name"][:40]] += 1
print("kernels > 1 ms:", dict(c))
if m:
    rows = [r for r in csv.DictReader(open(m[0])) if (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) > 1e6]
    print("memory copies > 1 ms:", [(r["Direction"], round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, 2)) for r in rows])
PY
HSA_ENABLE_SDMA=1 timeout -k 10 120 python3 -u tools/d2h_probe.py 2>&1 | grep -E "ms" | sed 's/^/SDMA=1 /'
