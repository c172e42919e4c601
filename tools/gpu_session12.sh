#!/bin/bash
# Session 12: A/B of the working tree (opaque-uniform SGPR fix, single staged
# path in run-time kernels, host PFA codelets) against HEAD and the PFA
# run-time variant, interleaved on one box.
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=spfft_amd/_native/variants
step t_all 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for rep in 1 2; do
for v in new head pfa; do
  lib=""; [ $v != new ] && lib=$V/libspfft_amd_$v.so
  for n in 256 240 200 180 100; do
    SPFFT_AMD_LIBRARY=$lib step ${v}_${n}_$rep 200 python bench.py --steps 40 --warmup 4 --size $n
  done
  SPFFT_AMD_LIBRARY=$lib step ${v}_240f_$rep 200 python bench.py --steps 40 --warmup 4 --size 240 --precision single
  SPFFT_AMD_LIBRARY=$lib step ${v}_240r_$rep 200 python bench.py --steps 40 --warmup 4 --size 240 --type r2c
done
done
step chk240 200 python bench.py --steps 2 --warmup 1 --size 240 --check
step chk256 200 python bench.py --steps 2 --warmup 1 --size 256 --check
step prof_240 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_240 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --size 240
for f in gpurun_out/*.log; do
  v=$(grep -o '"value": [0-9.]*' "$f" | head -1 | cut -d' ' -f2)
  e=$(grep -o '"check_error": {[^}]*}' "$f" | head -1)
  [ -n "$v" ] && echo "$(basename $f .log) $v $e"
done
true
