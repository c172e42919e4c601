#!/bin/bash
# kernel stats for the 512^3 configurations (R2C fp32 = BASELINE config 5 on one GPU; C2C fp64)
set -o pipefail
out=gpurun_out/${1:-r2_512}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for args in "--size 512 --type r2c --precision single" "--size 512 --type c2c" "--size 512 --type c2c --precision single"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p$i -o run -- python3 bench.py --steps 10 --warmup 2 --transforms 1 $args > $out/p$i.log 2>&1 || { tail $out/p$i.log; exit 1; }
  echo "== $args"; grep -o '"value": [0-9.]*' $out/p$i.log; python tools/kstats.py $out/p$i/run_kernel_stats.csv | head -6 | cut -c1-60,100-
done
