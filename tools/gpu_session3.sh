#!/bin/bash
# Session 3: full GPU test suite (incl. native runners + 2-rank RCCL probe),
# bench in both sync modes, rocprofv3 kernel stats for profiles/.
source tools/gpu_run.sh
step pytest_gpu 1200 python -m pytest tests -m gpu -q -p no:cacheprovider -x
step bench_stream 300 python bench.py --steps 200 --warmup 10
step bench_call 300 python bench.py --steps 200 --warmup 10 --sync call
step bench_r2c 300 python bench.py --steps 100 --warmup 10 --type r2c
step bench_128 300 python bench.py --steps 200 --warmup 10 --size 128
step bench_f32 300 python bench.py --steps 100 --warmup 10 --precision single
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof_c2c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3_c2c -o run --output-format csv -- python bench.py --steps 20 --warmup 3
step prof_r2c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3_r2c -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --type r2c
