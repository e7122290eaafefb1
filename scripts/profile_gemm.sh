#!/bin/bash
# rocprofv3 evidence for the projection GEMM (run on the GPU box via gpurun):
#   kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes.
#   scripts/profile_gemm.sh <tag> [shape,shape,...]
set -euo pipefail
TAG=$1
export IGR_TUNE_SHAPES=${2:-att_fwd_1m}
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 scripts/tune_gemm.py one current > "$OUT/trace.json" 2> "$OUT/trace.log"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 scripts/tune_gemm.py one current > "$OUT/fetch.json" 2> "$OUT/fetch.log"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 scripts/tune_gemm.py one current > "$OUT/write.json" 2> "$OUT/write.log"
python3 - "$OUT" <<'PY'
import csv, sys, glob, os
out = sys.argv[1]
def find(sub, name):
    return glob.glob(os.path.join(out, sub, '**', name), recursive=True)[0]
stats = list(csv.DictReader(open(find('trace', 'run_kernel_stats.csv'))))
for r in stats:
    if 'gemm' in r['Name']:
        print(f"{r['Name'][:70]:70s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:9.1f} us")
for sub, ctr in [('fetch', 'FETCH_SIZE'), ('write', 'WRITE_SIZE')]:
    rows = [r for r in csv.DictReader(open(find(sub, 'run_counter_collection.csv'))) if 'gemm_rows_persistent' in r['Kernel_Name']]
    vals = [float(r['Counter_Value']) for r in rows]
    print(ctr, 'per launch (KiB): n', len(vals), 'mean', sum(vals) / max(len(vals), 1))
PY
