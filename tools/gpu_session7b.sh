#!/bin/bash
# Session 7b: opt-in hipGraph replay in synchronous calls (C++ CLI, private
# stream): graphs on/off; graph test; full GPU suite.
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B=spfft_amd/_native/spfft_bench
step t_graph 300 python -u -m pytest tests/test_gpu_transform.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k graph
for n in 32 64 128 256; do
  r=3000; [ $n -eq 128 ] && r=1000; [ $n -eq 256 ] && r=200
  SPFFT_GRAPH=1 step cli_g1_$n 200 $B -d $n $n $n -r $r -o gpurun_out/cli_g1_$n.json -e compact -p gpu-gpu --cutoff 0.5 --warmup 20
  SPFFT_GRAPH=0 step cli_g0_$n 200 $B -d $n $n $n -r $r -o gpurun_out/cli_g0_$n.json -e compact -p gpu-gpu --cutoff 0.5 --warmup 20
done
step t_all 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
grep -h "transforms/s" gpurun_out/cli_*.log
true
