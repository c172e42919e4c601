#!/bin/bash
# Bench rate against the size of the y/x intermediate (SPFFT_INTER_BYTES): a
# capped intermediate runs the y and x stages plane range by plane range, each
# range's y output read back by its x stage while it is still in the
# Infinity Cache (and the other way round forward).
#   tools/inter_sweep.sh <out-dir> [bytes...]
set -o pipefail
out=${1:?out dir}
shift
mkdir -p "$out"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
SIZES=${*:-"0 16777216 33554432 67108864 134217728"}
CONFIGS=${SWEEP_CONFIGS:-"c2c256f64:--size=256,--precision=double c2c256f32:--size=256,--precision=single r2c512f32:--size=512,--type=r2c,--precision=single"}
for cfg in $CONFIGS; do
  name=${cfg%%:*}
  IFS=, read -r -a args <<< "${cfg#*:}"
  for b in $SIZES; do
    if [ "$b" = 0 ]; then unset SPFFT_INTER_BYTES; else export SPFFT_INTER_BYTES=$b; fi
    timeout -k 10 180 python3 bench.py --transforms 1 --steps 100 --warmup 10 --profile-reps 0 "${args[@]}" \
      > "$out/${name}_$b.log" 2>&1
    rc=$?
    [ $rc -ne 0 ] && { tail -5 "$out/${name}_$b.log"; exit $rc; }
    python3 -c 'import json,sys; r=json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0]); print(sys.argv[2], sys.argv[3], round(r["value"],1), round(r["ms_per_step"]*1e3,1), "us/pair")' \
      "$out/${name}_$b.log" "$name" "$b"
  done
done
unset SPFFT_INTER_BYTES
exit 0
