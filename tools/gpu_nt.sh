#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step chk_nt 300 python bench.py --steps 200 --warmup 5 --check
step prof_nt 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v3_nt -o run --output-format csv -- python bench.py --steps 10 --warmup 2
L=spfft_amd/_native/variants/libspfft_amd_nont.so
SPFFT_AMD_LIBRARY=$L step chk_nont 300 python bench.py --steps 200 --warmup 5 --check
SPFFT_AMD_LIBRARY=$L step prof_nont 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v3_nont -o run --output-format csv -- python bench.py --steps 10 --warmup 2
step chk_r2c 300 python bench.py --steps 100 --warmup 5 --check --type r2c
step chk_f32 300 python bench.py --steps 100 --warmup 5 --check --precision single
