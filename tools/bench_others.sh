#!/bin/bash
# bench.py lines of the other BASELINE configurations (one GPU): 128^3 C2C (B2) and
# 256^3 R2C (B3) at 4 and 1 transforms per step, 256^3 C2C with cutoff N/4.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
out=${1:-gpurun_out/others}; mkdir -p "$out"
for cfg in "b2_t4:--size 128" "b2_t1:--size 128 --transforms 1" "b3_t4:--size 256 --type r2c" \
           "b3_t1:--size 256 --type r2c --transforms 1" "c4_t4:--size 256 --cutoff 0.25"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 $args > "$out/$name.json" 2> "$out/$name.err" || { tail -5 "$out/$name.err"; exit 1; }
  echo "$name ($args): $(python3 -c 'import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(r["value"],1), r["vs_baseline"])' "$out/$name.json")"
done
