#!/bin/bash
# Compile-time mixed-radix engine (FftMR): correctness, then A/B against the run-time engine.
set -o pipefail
out=gpurun_out/mr
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_transform.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mixed_radix or composite" > $out/pytest.log 2>&1 || { tail -n 40 $out/pytest.log; exit 1; }
tail -n 2 $out/pytest.log
V=spfft_amd/_native/variants/libspfft_amd_nomr.so
lib() { [ "$1" = base ] && echo "" || echo "$V"; }
for v in base nomr; do
  SPFFT_AMD_LIBRARY=$(lib $v) timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$v -o run -- python3 bench.py --steps 20 --size 240 --transforms 1 > $out/prof_$v.log 2>&1 || exit 1
  echo "== $v"; python tools/kstats.py $out/prof_$v/run_kernel_stats.csv | head -6
done
for args in "--size 240 --transforms 1" "--size 200 --transforms 1" "--size 192 --transforms 1" "--size 240 --precision single --transforms 1" "--size 200 --precision single --transforms 1" "--size 240 --type r2c --transforms 1"; do
  for v in base nomr; do
    SPFFT_AMD_LIBRARY=$(lib $v) timeout -k 10 180 python bench.py $args > $out/b.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$out/b.json')); print('$args', '$v', round(d['value'],1))"
  done
done
