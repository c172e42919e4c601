#!/bin/bash
# y-stage LDS: no ColEntries reservation with column descriptors (the R2C x = 0 column
# gathers through the descriptor too). GPU tests, then A/B against the previous library.
source tools/gpu_run.sh
out=gpurun_out/ylds
mkdir -p $out
step tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
base=$GRAFT_REPO_ROOT/spfft_amd/_native/variants/libspfft_amd_base.so
for cfg in "256 c2c single 1 200" "256 c2c single 4 200" "256 r2c single 1 200" "512 r2c single 1 20" "256 r2c double 1 200" "256 c2c double 1 200" "128 c2c single 1 400"; do
  set -- $cfg
  for lib in new base new base; do
    if [ $lib = base ]; then export SPFFT_AMD_LIBRARY=$base; else unset SPFFT_AMD_LIBRARY; fi
    timeout -k 10 120 python bench.py --size $1 --type $2 --precision $3 --transforms $4 --steps $5 --warmup 3 > $out/r.json 2>/dev/null || exit 1
    echo "$cfg $lib $(python3 -c "import json;print(round(json.load(open('$out/r.json'))['value']))")"
  done
done
