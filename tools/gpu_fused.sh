#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step fz_small 300 python -m pytest tests/test_gpu_transform.py -m gpu -q -p no:cacheprovider -x -k "sphere_c2c_large or nan_poison"
step fz_bench 300 python bench.py --steps 100 --warmup 5 --check
step fz_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v11_fused -o run --output-format csv -- python bench.py --steps 10 --warmup 2
SPFFT_FUSED=0 step fz_off 300 python bench.py --steps 100 --warmup 5 --check
step fz_128 300 python bench.py --steps 100 --warmup 5 --check --size 128
step fz_512 300 python bench.py --steps 10 --warmup 2 --check --size 512
step fz_f32 300 python bench.py --steps 100 --warmup 5 --check --precision single
step fz_all 900 python -m pytest tests -m gpu -q -p no:cacheprovider
