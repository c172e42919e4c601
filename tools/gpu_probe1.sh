#!/bin/bash
# Roofline probes: HBM copy rates; stage kernels without FFT compute / exchanges.
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step hbm_copy 120 ./spfft_amd/_native/hbm_copy
for v in nocomp noexch; do
  L=spfft_amd/_native/variants/libspfft_amd_$v.so
  SPFFT_AMD_LIBRARY=$L step prof_$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p1_$v -o run --output-format csv -- python bench.py --steps 10 --warmup 2
done
