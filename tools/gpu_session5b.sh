#!/bin/bash
# In-place register-staged run-time engine (32 KB vs 64 KB LDS budget) vs the
# line-fast ping-pong engine of commit 60da0db; small sizes for launch overhead.
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=spfft_amd/_native/variants
step t_gpu 400 python -u -m pytest tests/test_gpu_transform.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for n in 240 200 180 100; do
  step rt32_$n 200 python bench.py --steps 40 --warmup 4 --size $n
  SPFFT_AMD_LIBRARY=$V/libspfft_amd_rt64k.so step rt64_$n 200 python bench.py --steps 40 --warmup 4 --size $n
  SPFFT_AMD_LIBRARY=$V/libspfft_amd_head.so step rtold_$n 200 python bench.py --steps 40 --warmup 4 --size $n
done
step rt32_240f 200 python bench.py --steps 40 --warmup 4 --size 240 --precision single
SPFFT_AMD_LIBRARY=$V/libspfft_amd_rt64k.so step rt64_240f 200 python bench.py --steps 40 --warmup 4 --size 240 --precision single
step rt32_240r 200 python bench.py --steps 40 --warmup 4 --size 240 --type r2c
step rt32_240chk 200 python bench.py --steps 4 --warmup 1 --size 240 --check
for n in 32 48 64; do
  step small_$n 200 python bench.py --steps 400 --warmup 20 --size $n
done
step prof_240 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_240 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --size 240
step prof_64 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_64 -o run --output-format csv -- python bench.py --steps 50 --warmup 2 --size 64
for f in gpurun_out/*.log; do
  v=$(grep -o '"value": [0-9.]*' "$f" | head -1)
  [ -n "$v" ] && echo "$(basename $f .log) $v"
done
true
