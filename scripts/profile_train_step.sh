#!/bin/bash
# rocprofv3 kernel trace of one training-step benchmark (run on the GPU box via gpurun):
#   scripts/profile_train_step.sh <tag> [bench_train.py arguments]
# prints the kernels by total time and leaves the stats csv under gpurun_out/prof_<tag>/.
set -euo pipefail
TAG=$1
shift
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 scripts/bench_train.py "$@" > "$OUT/step.json" 2> "$OUT/step.log"
python3 - "$OUT" <<'PY'
import csv, sys, glob, os
out = sys.argv[1]
f = glob.glob(os.path.join(out, 'trace', '**', 'run_kernel_stats.csv'), recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(open(os.path.join(out, 'step.json')).read().strip()[:300])
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:28]:
    print(f"{r['Name'][:90]:90s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us  {100*float(r['TotalDurationNs'])/tot:5.1f} %")
PY
