#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step pytest_tr 900 python -m pytest tests/test_gpu_transform.py -m gpu -q -p no:cacheprovider -x
step chk_c2c 300 python bench.py --steps 100 --warmup 5 --check
step chk_r2c 300 python bench.py --steps 100 --warmup 5 --check --type r2c
step chk_r512 300 python bench.py --steps 20 --warmup 3 --check --type r2c --precision single --size 512
step chk_c512d 300 python bench.py --steps 10 --warmup 2 --check --size 512
step prof_c2c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v7_c2c -o run --output-format csv -- python bench.py --steps 10 --warmup 2
step prof_r2c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v7_r2c -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --type r2c
step prof_r512 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v7_r512 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --type r2c --precision single --size 512
step prof_c512d 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v7_c512d -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --size 512
