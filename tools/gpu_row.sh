#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step pytest_tr 900 python -m pytest tests/test_gpu_transform.py -m gpu -q -p no:cacheprovider -x
for v in base norow; do
  if [ $v = base ]; then unset SPFFT_AMD_LIBRARY; else export SPFFT_AMD_LIBRARY=spfft_amd/_native/variants/libspfft_amd_$v.so; fi
  step chk_c2c_$v 300 python bench.py --steps 100 --warmup 5 --check
  step prof_c2c_$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v6_c2c_$v -o run --output-format csv -- python bench.py --steps 10 --warmup 2
  step prof_f32_$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v6_f32_$v -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --precision single
  step prof_r2c_$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v6_r2c_$v -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --type r2c
  step prof_r512_$v 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v6_r512_$v -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --type r2c --precision single --size 512
done
unset SPFFT_AMD_LIBRARY
step chk_f32 300 python bench.py --steps 100 --warmup 5 --check --precision single
step chk_r2c 300 python bench.py --steps 100 --warmup 5 --check --type r2c
step chk_r512 300 python bench.py --steps 20 --warmup 3 --check --type r2c --precision single --size 512
