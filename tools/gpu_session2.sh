#!/bin/bash
source tools/gpu_run.sh
step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
step bench1 300 python bench.py --steps 20 --warmup 3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof_stats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python bench.py --steps 10 --warmup 2
