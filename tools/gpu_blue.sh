#!/bin/bash
source tools/gpu_run.sh
step pytest_blue 900 python -m pytest tests/test_gpu_transform.py -m gpu -q -p no:cacheprovider -k "bluestein or sweep or r2c"
