#!/bin/bash
source tools/gpu_run.sh
step pytest_dist 900 python -m pytest tests/test_gpu_transform.py tests/test_torch_dist.py -m gpu -q -p no:cacheprovider -k "virtual or torch_dist"
