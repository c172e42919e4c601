#!/bin/bash
# Five more compile-time mixed-radix lengths (100, 108, 125, 135, 150): GPU tests of the
# MR kernels, then bench A/B against the previous library (variants/libspfft_amd_base.so).
source tools/gpu_run.sh
out=gpurun_out/mr2
mkdir -p $out
step tests 600 python -u -m pytest tests/test_gpu_transform.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "mixed_radix or c2c_sweep or r2c"
base=$GRAFT_REPO_ROOT/spfft_amd/_native/variants/libspfft_amd_base.so
for cfg in "100 c2c double" "108 c2c double" "125 c2c double" "135 c2c double" "150 c2c double" \
           "100 c2c single" "125 c2c single" "150 c2c single" "200 r2c double" "216 r2c double" "250 r2c double"; do
  set -- $cfg
  for lib in new base; do
    if [ $lib = base ]; then export SPFFT_AMD_LIBRARY=$base; else unset SPFFT_AMD_LIBRARY; fi
    timeout -k 10 120 python bench.py --size $1 --type $2 --precision $3 --transforms 1 --steps 300 --warmup 5 > $out/r.json 2>/dev/null || exit 1
    echo "$cfg $lib $(python3 -c "import json;print(round(json.load(open('$out/r.json'))['value']))")"
  done
done
