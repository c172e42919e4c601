#!/bin/bash
# Rehearsal of the driver's multi-rank bench launch on the 1-GPU box: ranks share
# the GPU, so the library picks the IPC peer-write data plane (RCCL refuses
# duplicate devices); everything else (torchrun env, gloo control plane, plan
# split, timing reduction, JSON line) is the multi-GPU path.
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
step d2 300 $L --nproc-per-node 2 --master-port 29541 bench.py --gpus 2 --steps 20 --warmup 3
step d4chk 300 $L --nproc-per-node 4 --master-port 29542 bench.py --gpus 4 --steps 10 --warmup 2 --check
step d2log 300 env SPFFT_LOG=1 $L --nproc-per-node 2 --master-port 29543 bench.py --gpus 2 --steps 4 --warmup 1 --size 64 --check
true
