#!/bin/bash
# Full GPU suite + smoke + headline bench after the batching / RCCL-fallback changes.
source tools/gpu_run.sh
out=gpurun_out/s3b
mkdir -p $out
step gpu_tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 180 python __graft_entry__.py smoke
step bench 300 python bench.py --steps 200 --warmup 10
