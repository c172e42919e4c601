#!/bin/bash
# A/B of kernel variant libraries on one box: interleaved bench runs + kernel stats.
# Usage: [BENCH_ARGS="--size 128"] bash tools/gpu_ab.sh <tag> <variant> [<variant> ...]   (variant "base" = default library)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
lib() { [ "$1" = base ] && echo "" || echo "spfft_amd/_native/variants/libspfft_amd_$1.so"; }
for v in "$@"; do
  SPFFT_AMD_LIBRARY=$(lib $v) timeout -k 10 120 python -m pytest tests -m gpu -x -q -k "sphere or virtual_ranks_distributions" > $out/pyt_$v.log 2>&1 || { echo "$v tests failed"; tail -n 20 $out/pyt_$v.log; exit 1; }
  SPFFT_AMD_LIBRARY=$(lib $v) timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$v -o run -- python3 bench.py --steps 20 $BENCH_ARGS > $out/prof_$v.log 2>&1 || exit 1
  echo "== $v"; python tools/kstats.py $out/prof_$v/run_kernel_stats.csv | head -6
done
for r in 1 2; do for v in "$@"; do
  SPFFT_AMD_LIBRARY=$(lib $v) timeout -k 10 120 python bench.py $BENCH_ARGS > $out/bench_${v}_$r.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open('$out/bench_${v}_$r.json')); print('$v', round(d['value'],1))"
done; done
