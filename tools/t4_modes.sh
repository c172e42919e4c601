#!/bin/bash
# Headline T = 4 execution modes on one box, alternated twice: multi_transform of 4
# transforms with batched launches on one stream (default), 4 per-transform streams,
# and T = 1 (profiles/r5/t4modes/summary.txt).
out=${1:-gpurun_out/t4modes}
mkdir -p "$out"
for round in 1 2; do
  for mode in batched per-transform t1; do
    env=""; args=""
    case $mode in
      per-transform) args="--streams per-transform" ;;
      t1) args="--transforms 1" ;;
    esac
    env $env timeout -k 10 200 python bench.py --steps 200 --warmup 10 --profile-reps 0 $args > "$out/${mode}_$round.json" 2>&1 || exit 1
    echo "$mode round$round $(grep '^{' "$out/${mode}_$round.json" | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["value"],1), round(r["ms_per_step"],4))')"
  done
done
