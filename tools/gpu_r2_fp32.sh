#!/bin/bash
set -o pipefail
out=gpurun_out/${1:-r2fp32}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for args in "--precision single" "--type r2c" "--type r2c --precision single"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p$i -o run -- python3 bench.py --steps 20 --transforms 1 $args > $out/p$i.log 2>&1 || { tail $out/p$i.log; exit 1; }
  echo "== $args"; grep -o '"value": [0-9.]*' $out/p$i.log; python tools/kstats.py $out/p$i/run_kernel_stats.csv | head -6 | cut -c1-60,100-
done
