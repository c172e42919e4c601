#!/bin/bash
# BASELINE config 5 path rehearsal on the 1-GPU box: 512^3 R2C fp32, 8 ranks (sharing the GPU:
# IPC peer-write data plane), every rank checks its round trip; plus the 4-rank 256^3 C2C case.
set -o pipefail
out=gpurun_out/${1:-r2c5}
mkdir -p $out
L="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 400 $L --nproc-per-node 8 --master-port 29571 bench.py --gpus 8 --size 512 --type r2c --precision single --transforms 1 --steps 3 --warmup 1 --check > $out/c5_np8.log 2>&1 || { tail -30 $out/c5_np8.log; exit 1; }
grep '"metric"' $out/c5_np8.log
timeout -k 10 300 $L --nproc-per-node 4 --master-port 29572 bench.py --gpus 4 --steps 5 --warmup 2 --check > $out/c4_np4.log 2>&1 || { tail -30 $out/c4_np4.log; exit 1; }
grep '"metric"' $out/c4_np4.log
