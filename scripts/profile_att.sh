#!/bin/bash
# rocprofv3 evidence for the attention edge kernels (run on the GPU box via gpurun):
#   kernel trace + stats of scripts/bench_att.py, then FETCH_SIZE and WRITE_SIZE in separate PMC passes.
#   scripts/profile_att.sh <tag>
set -euo pipefail
TAG=$1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 scripts/bench_att.py --steps 5 --warmup 1 > "$OUT/trace.json" 2> "$OUT/trace.log"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 scripts/bench_att.py --steps 2 --warmup 1 > "$OUT/fetch.json" 2> "$OUT/fetch.log"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 scripts/bench_att.py --steps 2 --warmup 1 > "$OUT/write.json" 2> "$OUT/write.log"
python3 - "$OUT" <<'PY'
import csv, sys, glob, os, collections
out = sys.argv[1]
def find(sub, name):
    return glob.glob(os.path.join(out, sub, '**', name), recursive=True)[0]
stats = list(csv.DictReader(open(find('trace', 'run_kernel_stats.csv'))))
for r in stats:
    if 'igr::' in r['Name']:
        print(f"{r['Name'][:80]:80s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e6:9.3f} ms")
for sub, ctr in [('fetch', 'FETCH_SIZE'), ('write', 'WRITE_SIZE')]:
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(find(sub, 'run_counter_collection.csv'))):
        if 'igr::' in r['Kernel_Name']:
            acc[r['Kernel_Name'][:60]].append(float(r['Counter_Value']))
    for k, v in acc.items():
        print(ctr, 'KiB per launch', k, 'n', len(v), 'mean', sum(v) / len(v))
PY
