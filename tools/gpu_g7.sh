#!/bin/bash
# T = 1..4 kernel splits; single-rank synchronous call trace (round 6)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/g7
AB_CONFIGS="t1:--transforms=1 t2:--transforms=2 t3:--transforms=3 t4:--transforms=4" timeout -k 10 900 bash tools/env_ab.sh gpurun_out/tsweep x=SPFFT_LOG=0 > gpurun_out/tsweep.log 2>&1
rc=$?; cat gpurun_out/tsweep.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/g7/sync -o run -- spfft_amd/_native/spfft_bench -d 128 128 128 -r 100 -m 1 -e compact -p gpu-gpu --cutoff 0.5 -o "" > gpurun_out/g7/sync.log 2>&1 || { tail gpurun_out/g7/sync.log; exit 1; }
python3 tools/ktimeline.py gpurun_out/g7/sync/run_kernel_trace.csv --skip 300 --tail 12
python3 tools/api_between.py gpurun_out/g7/sync/run_hip_api_trace.csv gpurun_out/g7/sync/run_kernel_trace.csv
