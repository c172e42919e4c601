#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step all_tests 1200 python -m pytest tests -m gpu -q -p no:cacheprovider
step b_c2c 300 python bench.py --steps 200 --warmup 10
step b_c2c_call 300 python bench.py --steps 200 --warmup 10 --sync call
step b_r2c 300 python bench.py --steps 200 --warmup 10 --type r2c
step b_f32 300 python bench.py --steps 200 --warmup 10 --precision single
step b_128 300 python bench.py --steps 200 --warmup 10 --size 128
step b_r512 300 python bench.py --steps 20 --warmup 3 --type r2c --precision single --size 512
step b_c025 300 python bench.py --steps 200 --warmup 10 --cutoff 0.25
step cli 300 ./spfft_amd/_native/spfft_bench -d 256 256 256 -r 50 -o gpurun_out/cli.json -e compact -p gpu-gpu --cutoff 0.5
