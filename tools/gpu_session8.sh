#!/bin/bash
# Session 8: batched LDS gather/scatter in the run-time and Bluestein engines and
# in the y/x copy-outs: GPU suite, then A/B against the previous commit (head).
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
H=spfft_amd/_native/variants/libspfft_amd_head.so
step t_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run_ab() {
  local tag=$1; shift
  step new_$tag 200 python bench.py "$@"
  SPFFT_AMD_LIBRARY=$H step old_$tag 200 python bench.py "$@"
}
run_ab 256 --steps 100 --warmup 5
run_ab 256r --steps 100 --warmup 5 --type r2c
run_ab 256f --steps 100 --warmup 5 --precision single
run_ab 128 --steps 200 --warmup 10 --size 128
for n in 240 200 180 100 60; do run_ab $n --steps 40 --warmup 4 --size $n; done
run_ab 240f --steps 40 --warmup 4 --size 240 --precision single
run_ab 210b --steps 20 --warmup 2 --size 202
step chk240 200 python bench.py --steps 2 --warmup 1 --size 240 --check
step prof_new 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_new -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --size 240
for f in gpurun_out/new_*.log; do
  t=$(basename $f .log); t=${t#new_}
  a=$(grep -o '"value": [0-9.]*' "$f" | head -1 | cut -d' ' -f2)
  b=$(grep -o '"value": [0-9.]*' gpurun_out/old_$t.log | head -1 | cut -d' ' -f2)
  echo "$t new=$a old=$b"
done
true
