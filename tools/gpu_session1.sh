#!/bin/bash
source tools/gpu_run.sh
step smoke 400 python __graft_entry__.py smoke
step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
step bench1 300 python bench.py --steps 20 --warmup 3
step bench_timing 300 python bench.py --steps 20 --warmup 3 --timing
