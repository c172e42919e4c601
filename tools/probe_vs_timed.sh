#!/bin/bash
# bench.py on 2 ranks sharing one GPU at 256^3, T = 1: the headline after the
# data-plane probe (every plane, or a subset) against no probe, per exchange type.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
out=${1:-gpurun_out/cmp}
mkdir -p "$out"
p=29800
for ex in ${EXCHANGES:-compact unbuffered}; do for probe in ${PROBES:-none rccl,ipc,relay}; do p=$((p+1))
  if [ "$probe" = none ]; then pa="--planes-probe 0"; else pa="--planes-probe 1 --probe-planes $probe"; fi
  f="$out/${ex}_${probe//,/-}.json"
  timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
    --master-port=$p bench.py --gpus 2 --steps ${STEPS:-100} --warmup 5 --size 256 --exchange $ex --transforms 1 \
    --profile-reps 0 $pa > "$f" 2> "${f%.json}.err" || { tail -5 "${f%.json}.err"; exit 1; }
  echo "$ex probe=$probe $(python3 -c 'import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(r["value"],1), round(r["ms_per_step"],4), {k: round(v["ms_per_step"],4) if "ms_per_step" in v else v for k, v in (r["config"].get("planes_ms") or {}).items()})' "$f")"
done; done
