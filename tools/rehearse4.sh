#!/bin/bash
# Multi-rank rehearsals on one GPU: 4 ranks through one RCCL communicator
# (virtual hosts, socket transport) and 2 ranks on the default plane, with the
# data-plane probe (planes_ms) and the measured peer copy rate in the record.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
out=${1:-gpurun_out/rehearse}
mkdir -p "$out"
SPFFT_RCCL_VIRTUAL_HOSTS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
  --master-addr=127.0.0.1 --master-port=29671 bench.py --gpus 4 --steps 10 --warmup 2 \
  > "$out/vh4.json" 2> "$out/vh4.err" || { tail -30 "$out/vh4.err"; exit 1; }
echo "vh4: $(tail -c 2500 "$out/vh4.json")"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr=127.0.0.1 --master-port=29672 bench.py --gpus 2 --steps 20 --warmup 3 \
  > "$out/ipc2.json" 2> "$out/ipc2.err" || { tail -30 "$out/ipc2.err"; exit 1; }
echo "ipc2: $(tail -c 2500 "$out/ipc2.json")"
