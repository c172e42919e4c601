#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof_stats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 10 --warmup 2
