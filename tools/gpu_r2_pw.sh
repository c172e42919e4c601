#!/bin/bash
# Plane-wave workload (H_loc psi, 64 bands) with batched multi_transform on/off.
source tools/gpu_run.sh
out=gpurun_out/pw
mkdir -p $out
step test 300 python -u -m pytest tests/test_models.py -q -p no:cacheprovider --timeout 120 --timeout-method thread
for cfg in "10 40" "20 30"; do
  set -- $cfg
  for T in 1 8; do
    for b in 0 1; do
      SPFFT_BATCH=$b timeout -k 10 120 python tools/pw_bench.py --alat $1 --ecut $2 --bands 64 --transforms $T > $out/r.json 2>/dev/null || exit 1
      cat $out/r.json
    done
  done
done
