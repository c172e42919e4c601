#!/bin/bash
# 4 ranks of spfft_bench (128^3, UNBUFFERED, synchronous calls) sharing the GPU,
# each under rocprofv3 (kernel + HIP API trace, one output per process), then a
# per-process kernel timeline and the host API calls between the kernels.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
out=${1:-gpurun_out/trace4}
rm -rf "$out"; mkdir -p "$out"
timeout -k 10 200 /opt/conda/bin/mpiexec -n 4 rocprofv3 --kernel-trace --hip-trace --output-format csv \
  -d "$out" -o "run_%pid%" -- spfft_amd/_native/spfft_bench -d 128 128 128 -r 50 -m 1 -e unbuffered \
  -p gpu-gpu --cutoff 0.5 -o "" > "$out/sb.log" 2>&1
rc=$?
grep transforms/s "$out/sb.log"
for f in $(find "$out" -name '*kernel_trace.csv' | sort); do
  echo "== $f"
  python3 tools/ktimeline.py "$f" --skip 200 --tail 14
  api=${f%kernel_trace.csv}hip_api_trace.csv
  [ -f "$api" ] && python3 tools/api_between.py "$api" "$f"
done
exit $rc
