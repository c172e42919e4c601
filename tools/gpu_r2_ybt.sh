#!/bin/bash
# y -> base LDS table (SPFFT_Y_BASE_TABLE=1 variant): GPU tests with the variant, then A/B.
source tools/gpu_run.sh
out=gpurun_out/ybt
mkdir -p $out
var=$GRAFT_REPO_ROOT/spfft_amd/_native/variants/libspfft_amd_ybt.so
export SPFFT_AMD_LIBRARY=$var
step tests 600 python -u -m pytest tests/test_gpu_transform.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "sweep or r2c or multi or mixed"
unset SPFFT_AMD_LIBRARY
for cfg in "256 c2c single 1 200" "256 c2c double 1 200" "256 c2c double 4 200" "512 r2c single 1 20" "256 r2c double 1 200"; do
  set -- $cfg
  for lib in ybt base ybt base; do
    if [ $lib = ybt ]; then export SPFFT_AMD_LIBRARY=$var; else unset SPFFT_AMD_LIBRARY; fi
    timeout -k 10 120 python bench.py --size $1 --type $2 --precision $3 --transforms $4 --steps $5 --warmup 3 > $out/r.json 2>/dev/null || exit 1
    echo "$cfg $lib $(python3 -c "import json;print(round(json.load(open('$out/r.json'))['value']))")"
  done
done
