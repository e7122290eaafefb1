#!/bin/bash
# Training through the trainer's DEFAULT configuration (no 'graph' key) at the shapes of
# BASELINE's small configurations: train_one_epoch() timed, ms per step = epoch / steps.
set -eo pipefail
out=${1:-gpurun_out/default_steps.jsonl}
: > "$out"
ml="--n-users 6040 --n-items 3706 --n-edges 1000000 --d 64 --epochs 5"
timeout -k 10 240 python -u scripts/bench_train.py $ml --layers 3 --model IGCN >> "$out"
timeout -k 10 240 python -u scripts/bench_train.py $ml --layers 2 --model IGCN >> "$out"
timeout -k 10 240 python -u scripts/bench_train.py $ml --layers 2 --model AttIGCN >> "$out"
timeout -k 10 240 python -u scripts/bench_train.py $ml --layers 3 --model LightGCN >> "$out"
timeout -k 10 240 python -u scripts/bench_train.py --n-users 29858 --n-items 40981 --n-edges 1030000 --d 128 --layers 3 --epochs 5 --model IGCN >> "$out"
