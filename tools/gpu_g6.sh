#!/bin/bash
# transforms-per-step sweep and single-rank call-mode costs (round 6)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/g6
for T in 4 8 2 4 8; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --transforms $T > gpurun_out/g6/b.json 2>/dev/null || exit 1
  echo "T=$T: $(python3 -c 'import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(r["value"],1), r["config"]["check_error"]["ok"])' gpurun_out/g6/b.json)"
done
for n in 128 256; do
  for mode in "" "--async"; do
    timeout -k 10 200 spfft_amd/_native/spfft_bench -d $n $n $n -r 100 -m 1 -e compact -p gpu-gpu --cutoff 0.5 -o "" $mode > gpurun_out/g6/sb.log 2>&1 || { tail gpurun_out/g6/sb.log; exit 1; }
    echo "spfft_bench 1 rank ${n}^3 $mode: $(grep transforms/s gpurun_out/g6/sb.log | tr -s ' ')"
  done
  SPFFT_GRAPH=1 timeout -k 10 200 spfft_amd/_native/spfft_bench -d $n $n $n -r 100 -m 1 -e compact -p gpu-gpu --cutoff 0.5 -o "" > gpurun_out/g6/sb.log 2>&1 || { tail gpurun_out/g6/sb.log; exit 1; }
  echo "spfft_bench 1 rank ${n}^3 graph: $(grep transforms/s gpurun_out/g6/sb.log | tr -s ' ')"
done
