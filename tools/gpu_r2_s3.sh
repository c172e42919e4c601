#!/bin/bash
# Round 2 session 3 validation: full GPU suite, smoke, headline bench, kernel stats.
source tools/gpu_run.sh
out=gpurun_out/s3
mkdir -p $out
step gpu_tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 180 python __graft_entry__.py smoke
step bench 300 python bench.py --steps 200 --warmup 10
step bench_t1 300 python bench.py --steps 200 --warmup 10 --transforms 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --steps 20 --transforms 1
python tools/kstats.py $out/prof/run_kernel_stats.csv > $out/kstats.txt 2>&1
cat $out/kstats.txt
