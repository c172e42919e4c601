#!/bin/bash
# Large-grid sub-batches: GPU tests, then 256^3 A/B over SPFFT_BATCH / SPFFT_BATCH_SPLIT
# and stream modes (3 runs each, transforms/s).
source tools/gpu_run.sh
out=gpurun_out/batch4
mkdir -p $out
step tests 300 python -u -m pytest tests/test_gpu_transform.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "multi_transform"
run() {
  local tag=$1; shift
  local vals=""
  for rep in 1 2 3; do
    env "$@" > $out/r.json 2>/dev/null || exit 1
    vals="$vals $(python3 -c "import json;print(round(json.load(open('$out/r.json'))['value']))")"
  done
  echo "$tag:$vals"
}
B="timeout -k 10 120 python bench.py --size 256 --steps 60 --warmup 5"
run "T4 streams unbatched" SPFFT_BATCH=0 $B --transforms 4
run "T4 streams split2" SPFFT_BATCH=1 $B --transforms 4
run "T4 streams split4" SPFFT_BATCH_SPLIT=4 $B --transforms 4
run "T8 streams unbatched" SPFFT_BATCH=0 $B --transforms 8
run "T8 streams split2" SPFFT_BATCH=1 $B --transforms 8
run "T8 streams split4" SPFFT_BATCH_SPLIT=4 $B --transforms 8
run "T4 sync-call unbatched" SPFFT_BATCH=0 $B --transforms 4 --sync call
run "T4 sync-call split2" SPFFT_BATCH=1 $B --transforms 4 --sync call
run "T4 one-stream batched" SPFFT_BATCH=1 $B --transforms 4 --streams one
