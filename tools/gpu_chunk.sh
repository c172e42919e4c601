#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SPFFT_CHUNK_PLANES=16 step pyt 300 python -m pytest tests -m gpu -x -q -p no:cacheprovider
for c in 0 8 16 32 64 128; do
SPFFT_CHUNK_PLANES=$c step bench_c$c 300 python bench.py --steps 30 --warmup 3
SPFFT_CHUNK_PLANES=$c step prof_c$c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c$c -o run --output-format csv -- python bench.py --steps 5 --warmup 2
done
