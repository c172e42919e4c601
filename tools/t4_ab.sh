#!/bin/bash
# Same-box A/B of run-time settings on the T = 4 (batched) bench lines: each setting
# alternated twice per configuration.
#   tools/t4_ab.sh <out-dir> <name>=<VAR=value,...> ...
set -o pipefail
out=${1:?out dir}
shift
mkdir -p "$out"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
CONFIGS=${AB_CONFIGS:-"f64:--size=256,--precision=double,--steps=200 f32:--size=256,--precision=single,--steps=200 r2c512:--size=512,--type=r2c,--precision=single,--steps=50"}
for round in 1 2; do
  for cfg in $CONFIGS; do
    cname=${cfg%%:*}
    IFS=, read -r -a args <<< "${cfg#*:}"
    for setting in "$@"; do
      name=${setting%%=*}
      IFS=, read -r -a envs <<< "${setting#*=}"
      log="$out/${name}_${cname}_$round.log"
      env "${envs[@]}" timeout -k 10 240 python3 bench.py --warmup 10 "${args[@]}" > "$log" 2>&1 || { tail -5 "$log"; exit 1; }
      echo "$name $cname round$round $(grep '^{' "$log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "transforms/s", round(d["ms_per_step"],4), "ms/step")')"
    done
  done
done
