#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in t2 t4; do
  SPFFT_AMD_LIBRARY=spfft_amd/_native/variants/libspfft_amd_$v.so step chk_$v 300 python bench.py --steps 100 --warmup 5 --check
  SPFFT_AMD_LIBRARY=spfft_amd/_native/variants/libspfft_amd_$v.so step prof_$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v10_$v -o run --output-format csv -- python bench.py --steps 10 --warmup 2
done
