#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof_base 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_base -o run --output-format csv -- python bench.py --steps 5 --warmup 2
for v in e8 e8b96; do
SPFFT_AMD_LIBRARY=spfft_amd/_native/variants/libspfft_amd_$v.so step pyt_$v 300 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "sphere"
SPFFT_AMD_LIBRARY=spfft_amd/_native/variants/libspfft_amd_$v.so step prof_$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$v -o run --output-format csv -- python bench.py --steps 5 --warmup 2
done
step bench 300 python bench.py --steps 30 --warmup 3
