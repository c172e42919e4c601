#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step pytest_gpu 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "sphere or c2c_sweep"
for ps in 0 8 16; do for pi in 0 8 16; do
  SPFFT_PAD_STICK=$ps SPFFT_PAD_INTER=$pi step prof_s${ps}_i${pi} 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s${ps}_i${pi} -o run --output-format csv -- python bench.py --steps 5 --warmup 2
done; done
