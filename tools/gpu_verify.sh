#!/bin/bash
source tools/gpu_run.sh
step pytest_all 1200 python -m pytest tests -m gpu -q -p no:cacheprovider
