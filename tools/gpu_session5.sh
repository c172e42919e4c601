#!/bin/bash
# Round-1 session 5: line-fast run-time engine (non-power-of-two sizes) vs the
# previous build, and the Infinity-Cache plane-chunk ring experiment.
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=spfft_amd/_native/variants
step t_gpu 400 python -u -m pytest tests/test_gpu_transform.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for n in 240 200 192 180; do
  step rt_new_$n 200 python bench.py --steps 40 --warmup 4 --size $n
  SPFFT_AMD_LIBRARY=$V/libspfft_amd_head.so step rt_old_$n 200 python bench.py --steps 40 --warmup 4 --size $n
done
step base 200 python bench.py --steps 100 --warmup 10
for c in 16 32 64; do
  SPFFT_CHUNK_PLANES=$c step chunk_$c 200 python bench.py --steps 100 --warmup 10
  SPFFT_CHUNK_PLANES=$c SPFFT_INTER_RING=1 step ring_$c 200 python bench.py --steps 100 --warmup 10
  SPFFT_AMD_LIBRARY=$V/libspfft_amd_ntinter0.so SPFFT_CHUNK_PLANES=$c SPFFT_INTER_RING=1 step ringt_$c 200 python bench.py --steps 100 --warmup 10
done
SPFFT_AMD_LIBRARY=$V/libspfft_amd_ntinter0.so SPFFT_CHUNK_PLANES=32 SPFFT_INTER_RING=1 step ringt_check 200 python bench.py --steps 10 --warmup 2 --check
SPFFT_AMD_LIBRARY=$V/libspfft_amd_ntinter0.so SPFFT_CHUNK_PLANES=32 SPFFT_INTER_RING=1 step prof_ringt 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ringt -o run --output-format csv -- python bench.py --steps 10 --warmup 2
step prof_240 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_240 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --size 240
for f in gpurun_out/*.log; do
  v=$(grep -o '"value": [0-9.]*' "$f" | head -1)
  [ -n "$v" ] && echo "$(basename $f .log) $v"
done
true
