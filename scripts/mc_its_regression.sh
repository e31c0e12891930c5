#!/bin/bash
# GPU box: configs[2] fused Monte-Carlo batch time against mean iterations over a p sweep
# (time = per-trial overhead + per-iteration cost x mean iterations).
set -u
for p in 0.04 0.05 0.06 0.065 0.07 0.075; do
  timeout -k 10 120 python3 scripts/diag/decode_launch.py --mc-bsc $p --warmup 1 --reps 3 | tail -1 || exit 1
done
