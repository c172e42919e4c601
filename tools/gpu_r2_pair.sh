#!/bin/bash
# Paired fp32 engine (SPFFT_F32_PAIR variant): full GPU test suite, then fp32 A/B.
set -o pipefail
out=gpurun_out/pair
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=spfft_amd/_native/variants/libspfft_amd_pair.so
SPFFT_AMD_LIBRARY=$V timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "single or long or float or True" --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -n 40 $out/pytest.log; exit 1; }
tail -n 3 $out/pytest.log
SPFFT_AMD_LIBRARY=$V timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_pair -o run -- python3 bench.py --steps 20 --precision single --transforms 1 > $out/prof_pair.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_base -o run -- python3 bench.py --steps 20 --precision single --transforms 1 > $out/prof_base.log 2>&1 || exit 1
for v in base pair; do echo "== $v"; python tools/kstats.py $out/prof_$v/run_kernel_stats.csv | head -8; done
lib() { [ "$1" = base ] && echo "" || echo "$V"; }
for args in "--precision single" "--precision single --transforms 1" "--precision single --type r2c --size 512 --steps 5" "--precision single --size 128"; do
  for r in 1; do for v in base pair; do
    SPFFT_AMD_LIBRARY=$(lib $v) timeout -k 10 180 python bench.py $args > $out/b.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$out/b.json')); print('$args', '$v', round(d['value'],1))"
  done; done
done
