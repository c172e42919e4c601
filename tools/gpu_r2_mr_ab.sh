#!/bin/bash
# FftMR shape variants: correctness subset, then per size/precision the kernel
# times (rocprofv3 kernel trace) and the bench value of the profiled run.
set -o pipefail
out=gpurun_out/mrab
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
lib() { [ "$1" = base ] && echo "" || echo "spfft_amd/_native/variants/libspfft_amd_$1.so"; }
for v in "$@"; do
  SPFFT_AMD_LIBRARY=$(lib $v) timeout -k 10 200 python -u -m pytest tests/test_gpu_transform.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mixed_radix" > $out/pyt_$v.log 2>&1 || { echo "$v tests failed"; tail -n 30 $out/pyt_$v.log; exit 1; }
done
for cfg in "240 double" "200 double" "192 double" "240 single" "200 single" "192 single"; do
  set -- $cfg; n=$1; p=$2; shift 2
  for v in $VARIANTS; do
    d=$out/p_${v}_${n}_$p
    SPFFT_AMD_LIBRARY=$(lib $v) timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps 20 --size $n --precision $p --transforms 1 > $d.json 2>$d.err || exit 1
    python tools/kstats_line.py $d/run_kernel_stats.csv $d.json "$n $p $v"
  done
done
