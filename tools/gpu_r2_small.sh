#!/bin/bash
# Small-grid probe: bench + kernel trace at 64^3 and 100^3 (4 transforms per step).
source tools/gpu_run.sh
out=gpurun_out/small
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for s in 64 100; do
  step b$s 120 python bench.py --size $s --steps 400 --warmup 20
  step p$s 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p$s -o run -- python3 bench.py --size $s --steps 100 --warmup 10
  python tools/kstats.py $out/p$s/run_kernel_stats.csv > $out/k$s.txt 2>&1
  cat $out/k$s.txt
done
