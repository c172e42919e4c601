#!/bin/bash
# relay plane tests, 2-rank bench with the plane probe, z-stage value-cache A/B (round 6)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/g2
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_torch_dist.py -k "relay" > gpurun_out/g2/relay.log 2>&1
rc=$?; tail -12 gpurun_out/g2/relay.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
  --master-port=29655 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/g2/bench2.json 2> gpurun_out/g2/bench2.err
rc=$?; tail -c 3000 gpurun_out/g2/bench2.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/g2/bench2.err; exit $rc; }
AB_CONFIGS="t4:--transforms=4 f32t4:--transforms=4,--precision=single" timeout -k 10 600 bash tools/env_ab.sh gpurun_out/zb2 zf0=SPFFT_NT_ZF=0 zf1=SPFFT_NT_ZF=1 > gpurun_out/zb2.log 2>&1
rc=$?; cat gpurun_out/zb2.log; for f in gpurun_out/zb2/split_*_1.txt; do echo "== $f"; grep "z_\|sum" $f; done; exit $rc
