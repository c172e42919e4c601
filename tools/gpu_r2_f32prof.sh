#!/bin/bash
# fp32 kernel stats: 256^3 C2C and 512^3 R2C (BASELINE config 5 on one GPU).
source tools/gpu_run.sh
out=gpurun_out/f32prof
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step b256 120 python bench.py --precision single --transforms 1 --steps 200 --warmup 5
step b512 200 python bench.py --precision single --type r2c --size 512 --transforms 1 --steps 20 --warmup 3
step p256 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p256 -o run -- python3 bench.py --precision single --transforms 1 --steps 20
step p512 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p512 -o run -- python3 bench.py --precision single --type r2c --size 512 --transforms 1 --steps 5 --warmup 2
python tools/kstats.py $out/p256/run_kernel_stats.csv
python tools/kstats.py $out/p512/run_kernel_stats.csv
