#!/bin/bash
# bench.py --transforms T at N=1, and a 2-rank rehearsal (ranks share the box's GPU).
set -o pipefail
out=gpurun_out/${1:-r2multi}
mkdir -p $out
for T in 1 2 4 1 2 4; do
  timeout -k 10 120 python bench.py --transforms $T > $out/t$T.json 2>$out/t$T.err || { cat $out/t$T.err | tail -20; exit 1; }
  python -c "import json; d=json.load(open('$out/t$T.json')); print('T=$T', round(d['value'],1))"
done
timeout -k 10 120 python bench.py --transforms 2 --check --steps 5 > $out/t2chk.json 2>&1 || { tail -20 $out/t2chk.json; exit 1; }
python -c "import json; d=json.load(open('$out/t2chk.json')); print('T=2 check', d['config']['check_error'])"
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 5 --warmup 2 --transforms 2 --check --size 128 > $out/np2.log 2>&1 || { tail -30 $out/np2.log; exit 1; }
grep metric $out/np2.log
