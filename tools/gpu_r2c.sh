#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step pytest_r2c 600 python -m pytest tests/test_gpu_transform.py -m gpu -q -p no:cacheprovider -k "r2c or R2C"
step chk_r2c 300 python bench.py --steps 100 --warmup 5 --check --type r2c
step prof_r2c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v5_r2c -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --type r2c
step chk_r2c_f32 300 python bench.py --steps 100 --warmup 5 --check --type r2c --precision single
step chk_r2c_512_f32 300 python bench.py --steps 20 --warmup 3 --check --type r2c --precision single --size 512
step prof_r2c_512_f32 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v5_r2c512 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --type r2c --precision single --size 512
