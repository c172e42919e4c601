#!/bin/bash
# 4 ranks on one GPU at 128^3 (IPC peer-write plane): bench.py stage times and
# spfft_bench rates under a few process settings. Output: <out>/*.json|log
out=${1:-gpurun_out/shared4}
mkdir -p "$out"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
MPIEXEC=$(command -v mpiexec || echo /opt/conda/bin/mpiexec)
port=29711
run_bench() {  # name nproc size T extra-env...
  local name=$1 np=$2 size=$3 T=$4; shift 4
  port=$((port + 1))
  env "$@" timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$np \
    --master-addr=127.0.0.1 --master-port=$port bench.py --gpus $np --steps 50 --warmup 5 \
    --size $size --transforms $T --exchange unbuffered > "$out/$name.json" 2> "$out/$name.err" \
    || { tail -20 "$out/$name.err"; exit 1; }
  echo "$name: $(python3 -c 'import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); st=r["config"]["stage_ms"]; print(round(r["value"],1), "transforms/s", round(r["ms_per_step"],3), "ms/step", {d: {k: round(v,3) for k,v in s.items()} for d,s in st.items()})' "$out/$name.json")"
}
run_bench b1_128 1 128 1
run_bench b2_128 2 128 1
run_bench b4_128 4 128 1
run_bench b4_128_q1 4 128 1 GPU_MAX_HW_QUEUES=1
run_bench b4_128_host 4 128 1 SPFFT_PEER_BARRIER=host
for m in 1 2; do
  for q in 4 1; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 "$MPIEXEC" -n 4 spfft_amd/_native/spfft_bench -d 128 128 128 -r 50 \
      -m $m -e all -p gpu-gpu --cutoff 0.5 -o "$out/sb4_m${m}_q$q.json" > "$out/sb4_m${m}_q$q.log" 2>&1 \
      || { tail -20 "$out/sb4_m${m}_q$q.log"; exit 1; }
    echo "spfft_bench 4 ranks -m $m queues $q: $(grep 'transforms/s' "$out/sb4_m${m}_q$q.log" | tr -s ' ' | tr '\n' ';')"
  done
done
exit 0
