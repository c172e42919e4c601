#!/bin/bash
# A/B of run-time knobs: each variant is "name:VAR=VAL[,VAR2=VAL2]" ("base" = no change).
# Usage: [BENCH_ARGS=...] bash tools/gpu_ab_env.sh <tag> base cm:SPFFT_INTER_CMAJOR=1
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
envof() { local spec=${1#*:}; [ "$spec" = "$1" ] && return; echo "${spec//,/ }"; }
nameof() { echo "${1%%:*}"; }
for v in "$@"; do
  n=$(nameof $v); e=$(envof $v)
  env $e timeout -k 10 200 python -m pytest tests -m gpu -x -q -k "sphere or virtual_ranks or r2c or poison" > $out/pyt_$n.log 2>&1 || { echo "$n tests failed"; tail -n 20 $out/pyt_$n.log; exit 1; }
  env $e timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$n -o run -- python3 bench.py --steps 20 --transforms 1 $BENCH_ARGS > $out/prof_$n.log 2>&1 || exit 1
  echo "== $n"; python tools/kstats.py $out/prof_$n/run_kernel_stats.csv | head -6 | cut -c1-50,100-
done
for r in 1 2; do for v in "$@"; do
  n=$(nameof $v); e=$(envof $v)
  env $e timeout -k 10 120 python bench.py $BENCH_ARGS > $out/bench_${n}_$r.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open('$out/bench_${n}_$r.json')); print('$n', round(d['value'],1))"
done; done
