#!/bin/bash
# rocprofv3 evidence for the bench's dominant kernel (run on the GPU box via gpurun).
#   1. kernel trace + stats   2. FETCH_SIZE pass   3. WRITE_SIZE pass (separate PMC passes)
# Outputs land in gpurun_out/prof_<tag>/; scripts/summarize_profile.py condenses them into profiles/.
set -euo pipefail
TAG=${1:-r01}
shift || true
ARGS=${@:---steps 10 --warmup 3 --cpu-passes 0}
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.log"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.log"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/write_bench.json" 2> "$OUT/write_bench.log"
echo "profile $TAG done"
