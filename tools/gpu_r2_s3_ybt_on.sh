#!/bin/bash
# Full GPU suite with the y -> base table on by default, smoke, headline and fp32 bench.
source tools/gpu_run.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 180 python __graft_entry__.py smoke
step bench 300 python bench.py --steps 200 --warmup 10
step bench_f32 300 python bench.py --steps 200 --warmup 10 --precision single --transforms 1
