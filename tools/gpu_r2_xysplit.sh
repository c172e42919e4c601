#!/bin/bash
# Two-stream y/x plane split (SPFFT_XY_SPLIT): correctness with every grid treated as
# large, then 256^3 A/B at 1 and 4 transforms per step (3 runs each).
source tools/gpu_run.sh
out=gpurun_out/xysplit
mkdir -p $out
export SPFFT_XY_SPLIT=1 SPFFT_BATCH_LARGE=0
step tests 600 python -u -m pytest tests/test_gpu_transform.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "sweep or r2c or mixed_radix or stream or multi"
unset SPFFT_XY_SPLIT SPFFT_BATCH_LARGE
run() {
  local tag=$1; shift
  local vals=""
  for rep in 1 2 3; do
    env "$@" > $out/r.json 2>/dev/null || exit 1
    vals="$vals $(python3 -c "import json;print(round(json.load(open('$out/r.json'))['value']))")"
  done
  echo "$tag:$vals"
}
B="timeout -k 10 120 python bench.py --size 256 --steps 100 --warmup 5"
run "T1 split0" SPFFT_XY_SPLIT=0 $B --transforms 1
run "T1 split1" SPFFT_XY_SPLIT=1 $B --transforms 1
run "T4 split0" SPFFT_XY_SPLIT=0 $B --transforms 4
run "T4 split1" SPFFT_XY_SPLIT=1 $B --transforms 4
run "T1 sync-call split0" SPFFT_XY_SPLIT=0 $B --transforms 1 --sync call
run "T1 sync-call split1" SPFFT_XY_SPLIT=1 $B --transforms 1 --sync call
run "T1 r2c split0" SPFFT_XY_SPLIT=0 $B --transforms 1 --type r2c
run "T1 r2c split1" SPFFT_XY_SPLIT=1 $B --transforms 1 --type r2c
