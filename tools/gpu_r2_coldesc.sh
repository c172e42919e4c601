#!/bin/bash
# Column descriptor with precomputed run origins: full GPU suite, then stage kernel times.
set -o pipefail
out=gpurun_out/coldesc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -n 40 $out/pytest.log; exit 1; }
tail -n 2 $out/pytest.log
for cfg in "256 double" "256 single" "240 double" "240 single" "128 double"; do
  set -- $cfg
  d=$out/p_$1_$2
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps 20 --size $1 --precision $2 --transforms 1 > $d.json 2>$d.err || exit 1
  python tools/kstats_line.py $d/run_kernel_stats.csv $d.json "$1 $2"
done
