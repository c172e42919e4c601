#!/bin/bash
# Session 11: prime-factor composite codelets (6, 10, 12, 15, 20) and the
# fewest-pass device radix planner vs the previous plans (oldrad).
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=spfft_amd/_native/variants
step t_comp 600 python -u -m pytest tests/test_gpu_transform.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "composite or sweep or bluestein or r2c"
for v in new oldrad; do
  lib=""; [ $v != new ] && lib=$V/libspfft_amd_$v.so
  for n in 240 200 180 120 100 60; do
    SPFFT_AMD_LIBRARY=$lib step ${v}_$n 200 python bench.py --steps 40 --warmup 4 --size $n
  done
  SPFFT_AMD_LIBRARY=$lib step ${v}_240f 200 python bench.py --steps 40 --warmup 4 --size 240 --precision single
  SPFFT_AMD_LIBRARY=$lib step ${v}_240r 200 python bench.py --steps 40 --warmup 4 --size 240 --type r2c
done
step chk240 200 python bench.py --steps 2 --warmup 1 --size 240 --check
step chk180r 200 python bench.py --steps 2 --warmup 1 --size 180 --check --type r2c
step t_all 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step prof_240 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_240 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --size 240
for f in gpurun_out/*.log; do
  v=$(grep -o '"value": [0-9.]*' "$f" | head -1 | cut -d' ' -f2)
  e=$(grep -o '"check_error": {[^}]*}' "$f" | head -1)
  [ -n "$v" ] && echo "$(basename $f .log) $v $e"
done
true
