#!/bin/bash
# rocprofv3 kernel trace of scripts/bench_train.py (run on the GPU box via gpurun):
#   scripts/profile_train.sh <tag> <bench_train.py args...>
# writes gpurun_out/prof_<tag>/ and prints the top kernels by total time.
set -euo pipefail
TAG=$1
shift
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 scripts/bench_train.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.log"
STATS=$(find "$OUT/trace" -name run_kernel_stats.csv -print -quit)
cp "$STATS" "$OUT/kernel_stats.csv"
cat "$OUT/bench.json"
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:28]:
    print(f"{r['Name'][:90]:90s} calls {int(r['Calls']):6d} avg {float(r['AverageNs'])/1e3:8.2f} us  {float(r['Percentage']):5.1f} %")
PY
