#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof_base 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v9_base -o run --output-format csv -- python bench.py --steps 10 --warmup 2
for v in b72 b100; do
  SPFFT_AMD_LIBRARY=spfft_amd/_native/variants/libspfft_amd_$v.so step chk_$v 300 python bench.py --steps 100 --warmup 5 --check
  SPFFT_AMD_LIBRARY=spfft_amd/_native/variants/libspfft_amd_$v.so step prof_$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v9_$v -o run --output-format csv -- python bench.py --steps 10 --warmup 2
done
for pi in 0 16 24; do
  SPFFT_PAD_INTER=$pi step prof_pi$pi 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v9_pi$pi -o run --output-format csv -- python bench.py --steps 10 --warmup 2
done
for ps in 0 16; do
  SPFFT_PAD_STICK=$ps step prof_ps$ps 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v9_ps$ps -o run --output-format csv -- python bench.py --steps 10 --warmup 2
done
