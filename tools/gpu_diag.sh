#!/bin/bash
source tools/gpu_run.sh
ldd spfft_amd/_native/libspfft_amd.so > gpurun_out/ldd.log 2>&1
step diag1 300 python -X faulthandler tools/diag1.py
