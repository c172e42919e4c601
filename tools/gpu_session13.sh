#!/bin/bash
# Session 13: per-precision composite radices (fp64 on, fp32 off) against HEAD.
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=spfft_amd/_native/variants
step t_all 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for v in new head; do
  lib=""; [ $v != new ] && lib=$V/libspfft_amd_$v.so
  for n in 256 240 200 180 120 100; do
    SPFFT_AMD_LIBRARY=$lib step ${v}_$n 200 python bench.py --steps 40 --warmup 4 --size $n
  done
  SPFFT_AMD_LIBRARY=$lib step ${v}_240f 200 python bench.py --steps 40 --warmup 4 --size 240 --precision single
  SPFFT_AMD_LIBRARY=$lib step ${v}_256f 200 python bench.py --steps 40 --warmup 4 --size 256 --precision single
  SPFFT_AMD_LIBRARY=$lib step ${v}_240r 200 python bench.py --steps 40 --warmup 4 --size 240 --type r2c
  SPFFT_AMD_LIBRARY=$lib step ${v}_256r 200 python bench.py --steps 40 --warmup 4 --size 256 --type r2c
done
step chk240 200 python bench.py --steps 2 --warmup 1 --size 240 --check
step chk180r 200 python bench.py --steps 2 --warmup 1 --size 180 --check --type r2c
step chk240f 200 python bench.py --steps 2 --warmup 1 --size 240 --check --precision single
step smoke 200 python __graft_entry__.py smoke
step bench_default 300 python bench.py
step prof_240 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_240 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --size 240
for f in gpurun_out/*.log; do
  v=$(grep -o '"value": [0-9.]*' "$f" | head -1 | cut -d' ' -f2)
  e=$(grep -o '"check_error": {[^}]*}' "$f" | head -1)
  [ -n "$v" ] && echo "$(basename $f .log) $v $e"
done
true
