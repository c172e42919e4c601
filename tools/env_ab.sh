#!/bin/bash
# Same-box A/B of run-time settings: per-kernel stats of bench.py (one transform per
# step) under each setting, the settings alternated twice.
#   tools/env_ab.sh <out-dir> <name>=<VAR=value,VAR2=value> ...
# e.g. tools/env_ab.sh gpurun_out/ab off=SPFFT_Y_PIPE=0 on=SPFFT_Y_PIPE=1
set -o pipefail
out=${1:?out dir}
shift
mkdir -p "$out"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
CONFIGS=${AB_CONFIGS:-"f64:--size=256,--precision=double f32:--size=256,--precision=single r2c512:--size=512,--type=r2c,--precision=single"}
for round in 1 2; do
  for setting in "$@"; do
    name=${setting%%=*}
    IFS=, read -r -a envs <<< "${setting#*=}"
    for cfg in $CONFIGS; do
      cname=${cfg%%:*}
      IFS=, read -r -a args <<< "${cfg#*:}"
      d="$out/${name}_${cname}_$round"
      env "${envs[@]}" timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run \
        -- python3 bench.py --transforms 1 --steps 30 --warmup 5 --profile-reps 0 "${args[@]}" > "$d.log" 2>&1
      rc=$?
      [ $rc -ne 0 ] && { tail -5 "$d.log"; exit $rc; }
      python3 tools/ktrace_split.py "$d/run_kernel_trace.csv" > "$out/split_${name}_${cname}_$round.txt"
      rate=$(grep '^{' "$d.log" | python3 -c 'import json,sys; print(round(json.loads(sys.stdin.read())["value"],1))')
      echo "$name $cname round$round rate=$rate $(tail -1 "$out/split_${name}_${cname}_$round.txt")"
    done
  done
done
exit 0
