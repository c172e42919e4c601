#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step fz_small 300 python -m pytest tests/test_gpu_transform.py -m gpu -q -p no:cacheprovider -x -k "sphere_c2c_large or nan_poison"
for cfg in "1 3" "2 4" "3 5" "4 6" "2 8"; do
  set -- $cfg
  SPFFT_FUSED_LAG=$1 SPFFT_FUSED_RING=$2 step prof_L$1R$2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v12_L$1R$2 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --check
done
