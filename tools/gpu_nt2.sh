#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step chk_base 300 python bench.py --steps 200 --warmup 5 --check
step prof_base 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v4_base -o run --output-format csv -- python bench.py --steps 10 --warmup 2
L=spfft_amd/_native/variants/libspfft_amd_ntv.so
SPFFT_AMD_LIBRARY=$L step chk_ntv 300 python bench.py --steps 200 --warmup 5 --check
SPFFT_AMD_LIBRARY=$L step prof_ntv 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v4_ntv -o run --output-format csv -- python bench.py --steps 10 --warmup 2
step chk_r2c 300 python bench.py --steps 100 --warmup 5 --check --type r2c
step prof_r2c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v4_r2c -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --type r2c
step prof_f32 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v4_f32 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --precision single
