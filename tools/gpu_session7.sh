#!/bin/bash
# Session 7: hipGraph whole-direction replay (single rank): tests, call/stream
# mode with graphs on/off at small and headline sizes.
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step t_graph 300 python -u -m pytest tests/test_gpu_transform.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "graph or sweep or r2c or stream"
for n in 32 64 128 256; do
  st=400; [ $n -eq 256 ] && st=200
  step g1call_$n 200 python bench.py --steps $st --warmup 20 --size $n --sync call
  SPFFT_GRAPH=0 step g0call_$n 200 python bench.py --steps $st --warmup 20 --size $n --sync call
  step g1strm_$n 200 python bench.py --steps $st --warmup 20 --size $n
  SPFFT_GRAPH=0 step g0strm_$n 200 python bench.py --steps $st --warmup 20 --size $n
done
step chk 200 python bench.py --steps 4 --warmup 2 --check
step t_all 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for f in gpurun_out/*.log; do
  v=$(grep -o '"value": [0-9.]*' "$f" | head -1)
  [ -n "$v" ] && echo "$(basename $f .log) $v"
done
true
