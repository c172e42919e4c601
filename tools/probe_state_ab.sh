#!/bin/bash
# 2 ranks sharing one GPU, 256^3 COMPACT, T = 1: the ipc headline after a relay-plane
# probe, with the in-tree library and with each variant library (name=path).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
out=${1:?out}; shift
mkdir -p "$out"
p=29950
for setting in base "$@"; do
  name=${setting%%=*}; lib=${setting#*=}
  if [ "$name" = base ]; then unset SPFFT_AMD_LIBRARY; else export SPFFT_AMD_LIBRARY=$lib; fi
  for probe in none relay; do p=$((p+1))
    if [ "$probe" = none ]; then pa="--planes-probe 0"; else pa="--planes-probe 1 --probe-planes $probe"; fi
    f="$out/${name}_$probe.json"
    timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
      --master-port=$p bench.py --gpus 2 --steps 100 --warmup 5 --size 256 --exchange compact --transforms 1 \
      --profile-reps 0 --plane ipc $pa > "$f" 2> "${f%.json}.err" || { tail -5 "${f%.json}.err"; exit 1; }
    echo "$name probe=$probe $(python3 -c 'import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(r["value"],1))' "$f")"
  done
done
