#!/bin/bash
# Batched multi-transform timeline: kernel trace of bench.py at 64^3 / 256^3, T=4, batched.
source tools/gpu_run.sh
out=gpurun_out/batch2
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step t1_64 120 python bench.py --size 64 --transforms 1 --steps 400 --warmup 5
step t1_256 120 python bench.py --size 256 --transforms 1 --steps 60 --warmup 5
step p64 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p64 -o run -- python3 bench.py --size 64 --steps 50 --warmup 5
step p256 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p256 -o run -- python3 bench.py --size 256 --steps 10 --warmup 2
python tools/kstats.py $out/p64/run_kernel_stats.csv
python tools/kstats.py $out/p256/run_kernel_stats.csv
