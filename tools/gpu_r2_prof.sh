#!/bin/bash
# Round 2 profiling step: headline bench + kernel-trace stats (csv) + a GPU test subset.
# Usage (on the GPU box): bash tools/gpu_r2_prof.sh <tag> [pytest -k expr]
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
if [ -n "$2" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$2" > $out/pytest.log 2>&1 || { tail -n 30 $out/pytest.log; exit 1; }
  tail -n 2 $out/pytest.log
fi
timeout -k 10 120 python bench.py > $out/bench.json 2> $out/bench.err || exit 1
cat $out/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --steps 20 > $out/prof.log 2>&1 || exit 1
python tools/kstats.py $out/prof/run_kernel_stats.csv
