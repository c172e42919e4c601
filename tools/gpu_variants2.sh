#!/bin/bash
# Kernel variants: LF stride fix, direct row stores in x/y backward.
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step chk_base 300 python bench.py --steps 100 --warmup 5 --check
step prof_base 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v2_base -o run --output-format csv -- python bench.py --steps 10 --warmup 2
for v in nofix xd yd xyd; do
  L=spfft_amd/_native/variants/libspfft_amd_$v.so
  SPFFT_AMD_LIBRARY=$L step chk_$v 300 python bench.py --steps 100 --warmup 5 --check
  SPFFT_AMD_LIBRARY=$L step prof_$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v2_$v -o run --output-format csv -- python bench.py --steps 10 --warmup 2
done
