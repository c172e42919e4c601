#!/bin/bash
# distributed GPU tests + 2-rank bench with the plane autotune (round 6)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/g5
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
  --master-port=29681 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/g5/bench2.json 2> gpurun_out/g5/bench2.err
rc=$?; [ $rc -ne 0 ] && { tail -30 gpurun_out/g5/bench2.err; exit $rc; }
python3 -c 'import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=r["config"]; print(round(r["value"],1), c["data_plane"], json.dumps(c["plane_choice"]), json.dumps(c["planes_ms"]))' gpurun_out/g5/bench2.json
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_torch_dist.py tests/test_native_programs.py > gpurun_out/g5/tdist.log 2>&1
rc=$?; tail -5 gpurun_out/g5/tdist.log; [ $rc -ne 0 ] && { grep -m3 -A30 "FAILED\|Error" gpurun_out/g5/tdist.log | head -80; }
exit $rc
