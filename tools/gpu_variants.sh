#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step base_spin 300 python bench.py --steps 30 --warmup 3
SPFFT_SYNC=block step base_block 300 python bench.py --steps 30 --warmup 3
for v in 48 96 128; do
  SPFFT_AMD_LIBRARY=spfft_amd/_native/variants/libspfft_amd_b$v.so step var_b$v 300 python bench.py --steps 30 --warmup 3
  SPFFT_AMD_LIBRARY=spfft_amd/_native/variants/libspfft_amd_b$v.so step prof_b$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b$v -o run --output-format csv -- python bench.py --steps 5 --warmup 2
done
step prof_base 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_base -o run --output-format csv -- python bench.py --steps 5 --warmup 2
