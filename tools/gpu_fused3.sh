#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SPFFT_FUSED_DEBUG=1 step prof_nowait 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v13_nowait -o run --output-format csv -- python bench.py --steps 10 --warmup 2
SPFFT_FUSED_DEBUG=1 SPFFT_FUSED_RING=8 SPFFT_FUSED_LAG=1 step prof_nowait8 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v13_nowait8 -o run --output-format csv -- python bench.py --steps 10 --warmup 2
