#!/bin/bash
# peer-plane natural stick layout: IPC tests, fuzz, 2-rank trace (round 6)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/g9
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_torch_dist.py -k "ipc or fuzz or bench or exchange_failure" tests/test_gpu_transform.py -k "ipc or virtual or UNBUFFERED or unbuffered or peer or fuzz" > gpurun_out/g9/tests.log 2>&1
rc=$?; tail -3 gpurun_out/g9/tests.log; [ $rc -ne 0 ] && { grep -m3 -A30 "FAILED\|Error" gpurun_out/g9/tests.log | head -60; exit $rc; }
bash tools/trace_shared2.sh gpurun_out/g9/trace2 > gpurun_out/g9/trace2.log 2>&1
rc=$?; grep -A8 "== rank\|^{" gpurun_out/g9/trace2.log | head -40; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
  --master-port=29695 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/g9/bench2.json 2> gpurun_out/g9/bench2.err || { tail -20 gpurun_out/g9/bench2.err; exit 1; }
python3 -c 'import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=r["config"]; print(round(r["value"],1), c["data_plane"], c["check_error"]["roundtrip"], json.dumps(c["stage_ms"]))' gpurun_out/g9/bench2.json
