#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step pytest_tr 900 python -m pytest tests/test_gpu_transform.py -m gpu -q -p no:cacheprovider -x
step chk_c2c 300 python bench.py --steps 200 --warmup 5 --check
step chk_r512 300 python bench.py --steps 20 --warmup 3 --check --type r2c --precision single --size 512
step chk_f32 300 python bench.py --steps 100 --warmup 5 --check --precision single
step prof_r512 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v8_r512 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --type r2c --precision single --size 512
step prof_f32 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v8_f32 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --precision single
