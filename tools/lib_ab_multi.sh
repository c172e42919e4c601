#!/bin/bash
# Same-box A/B of library builds on the multi-rank single-GPU paths: bench.py on
# 2 ranks at 256^3 (COMPACT and UNBUFFERED, IPC peer-write plane) and 1 rank, for
# each library (name=path; "base" = the in-tree build), two alternated rounds.
#   tools/lib_ab_multi.sh <out-dir> name=lib.so ...
set -o pipefail
out=${1:?out dir}; shift
mkdir -p "$out"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
port=29711
for round in 1 2; do
  for setting in base "$@"; do
    name=${setting%%=*}
    lib=${setting#*=}
    if [ "$name" = base ]; then unset SPFFT_AMD_LIBRARY; else export SPFFT_AMD_LIBRARY=$lib; fi
    for cfg in 2:compact:1 2:unbuffered:1 2:compact:4 1:compact:4; do
      IFS=: read -r np ex t <<< "$cfg"
      port=$((port + 1))
      f="$out/${name}_${np}r_${ex}_t${t}_$round.json"
      timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$np \
        --master-addr=127.0.0.1 --master-port=$port bench.py --gpus $np --steps 40 --warmup 5 \
        --size 256 --exchange $ex --transforms $t --profile-reps 0 > "$f" 2> "${f%.json}.err" \
        || { tail -20 "${f%.json}.err"; exit 1; }
      echo "$name round$round ${np}r $ex T=$t: $(python3 -c 'import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(r["value"],1), r["config"]["data_plane"], r["config"]["check_error"]["ok"])' "$f")"
    done
  done
done
unset SPFFT_AMD_LIBRARY
exit 0
