#!/bin/bash
# Training-step timings on one GPU: ML-1M shape (IGCN / AttIGCN / LightGCN, eager and
# hipGraph), Gowalla shape and 1 M x 100 K x 20 M.  One JSON line per run.
set -eo pipefail
out=${1:-gpurun_out/train_steps.jsonl}
: > "$out"
ml="--n-users 6040 --n-items 3706 --n-edges 1000000 --d 64 --layers 2 --steps 200 --warmup 20"
for m in IGCN AttIGCN LightGCN; do
  echo "== $m ML-1M graph" >&2
  timeout -k 10 240 python -u scripts/bench_train.py $ml --model $m --graph >> "$out"
  echo "== $m ML-1M eager" >&2
  timeout -k 10 240 python -u scripts/bench_train.py $ml --model $m >> "$out"
done
echo "== IGCN gowalla graph" >&2
timeout -k 10 240 python -u scripts/bench_train.py --n-users 29858 --n-items 40981 --n-edges 1030000 --d 128 --layers 3 --steps 200 --warmup 20 --graph >> "$out"
echo "== IGCN 1Mx100K" >&2
timeout -k 10 400 python -u scripts/bench_train.py --steps 30 --warmup 5 >> "$out"
