#!/bin/bash
# Several ranks on one GPU (IPC peer-write plane): bench.py on 2 ranks at 256^3
# (UNBUFFERED and COMPACT) and spfft_bench on 4 ranks at 128^3 (-e all), under
# each setting of SPFFT_STAGE_RELEASE (1 = a system-scope release at the end of
# every storing wave, the round-5 form; 0 = the barrier round's per-XCD
# write-back only). Output: <out>/<name>_*.json
#   tools/shared_gpu_ab.sh <out-dir> [settings...]   (default: 0 1)
out=${1:-gpurun_out/shared_gpu}
shift
settings=${*:-0 1}
mkdir -p "$out"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
MPIEXEC=$(command -v mpiexec || echo /opt/conda/bin/mpiexec)
port=29611
for rel in $settings; do
  for ex in unbuffered compact; do
    port=$((port + 1))
    SPFFT_STAGE_RELEASE=$rel timeout -k 10 150 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=$port bench.py --gpus 2 \
      --steps 20 --warmup 3 --size 256 --exchange $ex --transforms 1 \
      > "$out/rel${rel}_2r256_${ex}.json" 2> "$out/rel${rel}_2r256_${ex}.err" || { tail -20 "$out/rel${rel}_2r256_${ex}.err"; exit 1; }
    echo "rel=$rel 2 ranks 256^3 $ex: $(python3 -c 'import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(r["value"],1), "transforms/s", r["config"]["check_error"]["roundtrip"], r["config"]["data_plane"])' "$out/rel${rel}_2r256_${ex}.json")"
  done
  SPFFT_STAGE_RELEASE=$rel timeout -k 10 200 "$MPIEXEC" -n 4 spfft_amd/_native/spfft_bench -d 128 128 128 -r 20 \
    -m 2 -e all -p gpu-gpu --cutoff 0.5 -o "$out/rel${rel}_4r128.json" > "$out/rel${rel}_4r128.log" 2>&1 \
    || { tail -20 "$out/rel${rel}_4r128.log"; exit 1; }
  echo "rel=$rel 4 ranks 128^3: $(grep -i 'transforms/s' "$out/rel${rel}_4r128.log" | tr '\n' ' ')"
done
exit 0
