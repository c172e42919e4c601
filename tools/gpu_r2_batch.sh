#!/bin/bash
# Batched multi-transform: GPU tests, then A/B (SPFFT_BATCH=0/1) of bench.py with T
# transforms per step on one shared stream (--streams one) and on private streams
# (--sync call), plus the default per-transform streams for reference.
source tools/gpu_run.sh
out=gpurun_out/batch
mkdir -p $out
step tests 300 python -u -m pytest tests/test_gpu_transform.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "multi_transform"
for s in 64 100 128 256; do
  st=400; [ $s -ge 256 ] && st=60
  for T in 4 8; do
    for mode in "--streams one" "--sync call"; do
      for b in 0 1; do
        SPFFT_BATCH=$b timeout -k 10 120 python bench.py --size $s --transforms $T --steps $st --warmup 5 $mode > $out/r.json 2>/dev/null || exit 1
        python3 -c "import json;d=json.load(open('$out/r.json'));print('size $s T=$T $mode batch=$b', round(d['value']))"
      done
    done
  done
  timeout -k 10 120 python bench.py --size $s --transforms 4 --steps $st --warmup 5 > $out/r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$out/r.json'));print('size $s T=4 per-transform streams', round(d['value']))"
done
