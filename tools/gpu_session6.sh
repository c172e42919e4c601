#!/bin/bash
# Session 6: confirm the committed in-place run-time engine build (GPU tests,
# headline bench, non-power-of-two sizes, sync-call small sizes) + kernel stats.
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step t_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step b256 200 python bench.py --steps 200 --warmup 10
step b256chk 200 python bench.py --steps 4 --warmup 1 --check
step b240 200 python bench.py --steps 40 --warmup 4 --size 240
step b240f 200 python bench.py --steps 40 --warmup 4 --size 240 --precision single
for n in 32 64 128; do
  step call_$n 200 python bench.py --steps 400 --warmup 20 --size $n --sync call
  step strm_$n 200 python bench.py --steps 400 --warmup 20 --size $n
done
step prof_256 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_256 -o run --output-format csv -- python bench.py --steps 10 --warmup 2
for f in gpurun_out/*.log; do
  v=$(grep -o '"value": [0-9.]*' "$f" | head -1)
  [ -n "$v" ] && echo "$(basename $f .log) $v"
done
true
