#!/bin/bash
# 4 ranks sharing one GPU at 128^3 (bench.py, stream-ordered) for the in-tree library
# and each variant (name=path), two alternated rounds.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
out=${1:?out}; shift
mkdir -p "$out"
p=29400
for round in 1 2; do
  for setting in base "$@"; do
    name=${setting%%=*}; lib=${setting#*=}
    if [ "$name" = base ]; then unset SPFFT_AMD_LIBRARY; else export SPFFT_AMD_LIBRARY=$lib; fi
    for cfg in ${CFGS:-unbuffered:1 compact:1 unbuffered:4}; do
      IFS=: read -r ex t <<< "$cfg"; p=$((p+1))
      f="$out/${name}_${ex}_t${t}_$round.json"
      timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr=127.0.0.1 \
        --master-port=$p bench.py --gpus 4 --steps 100 --warmup 5 --size 128 --exchange $ex --transforms $t \
        --profile-reps 0 --planes-probe 0 --plane ipc > "$f" 2> "${f%.json}.err" || { tail -5 "${f%.json}.err"; exit 1; }
      echo "$name round$round $ex T=$t $(python3 -c 'import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(r["value"],1))' "$f")"
    done
  done
done
