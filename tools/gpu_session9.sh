#!/bin/bash
# Session 9: run-time engine workgroup size (256 / 512 / 1024 threads, 64 or
# 128 KB) at non-power-of-two sizes; quick correctness of each variant.
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=spfft_amd/_native/variants
for v in base t512 t1024 t512e8k; do
  lib=""; [ $v != base ] && lib=$V/libspfft_amd_$v.so
  SPFFT_AMD_LIBRARY=$lib step chk_$v 200 python bench.py --steps 2 --warmup 1 --size 120 --check
  for n in 240 200 180 100; do
    SPFFT_AMD_LIBRARY=$lib step ${v}_$n 200 python bench.py --steps 40 --warmup 4 --size $n
  done
  SPFFT_AMD_LIBRARY=$lib step ${v}_240f 200 python bench.py --steps 40 --warmup 4 --size 240 --precision single
  SPFFT_AMD_LIBRARY=$lib step ${v}_240r 200 python bench.py --steps 40 --warmup 4 --size 240 --type r2c
done
for f in gpurun_out/*.log; do
  v=$(grep -o '"value": [0-9.]*' "$f" | head -1 | cut -d' ' -f2)
  e=$(grep -o '"check_error": {[^}]*}' "$f" | head -1)
  echo "$(basename $f .log) $v $e"
done
true
