#!/bin/bash
# Last GPU call of session 3: multi_transform / plane-wave tests, the y base-table A/B,
# then the README performance table.
source tools/gpu_run.sh
step tests 300 python -u -m pytest tests/test_gpu_transform.py tests/test_models.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "multi_transform or planewave"
bash tools/gpu_r2_ybt.sh || exit 1
bash tools/gpu_r2_table.sh r2s3table
