#!/bin/bash
# Compile-time mixed-radix lengths 48, 60, 72, 80, 90: GPU tests, then bench A/B
# against the previous library (variants/libspfft_amd_base.so).
source tools/gpu_run.sh
out=gpurun_out/mr3
mkdir -p $out
step tests 600 python -u -m pytest tests/test_gpu_transform.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "mixed_radix or c2c_sweep or r2c"
base=$GRAFT_REPO_ROOT/spfft_amd/_native/variants/libspfft_amd_base.so
for cfg in "48 c2c double 4" "60 c2c double 4" "72 c2c double 4" "80 c2c double 4" "90 c2c double 4" \
           "96 r2c double 1" "120 r2c double 1" "144 r2c double 1" "160 r2c double 1" "180 r2c double 1" \
           "180 r2c single 1"; do
  set -- $cfg
  for lib in new base; do
    if [ $lib = base ]; then export SPFFT_AMD_LIBRARY=$base; else unset SPFFT_AMD_LIBRARY; fi
    timeout -k 10 120 python bench.py --size $1 --type $2 --precision $3 --transforms $4 --steps 300 --warmup 5 > $out/r.json 2>/dev/null || exit 1
    echo "$cfg $lib $(python3 -c "import json;print(round(json.load(open('$out/r.json'))['value']))")"
  done
done
