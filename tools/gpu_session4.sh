#!/bin/bash
# Session 4: IPC peer-write data plane (multi-process ranks sharing the GPU).
source tools/gpu_run.sh
step pytest_ipc 600 python -m pytest tests/test_torch_dist.py tests/test_gpu_transform.py -m gpu -q -p no:cacheprovider -x
step bench1 300 python bench.py --steps 200 --warmup 10
step bench_2rank_shared 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 50 --warmup 5
step bench_2rank_unbuf 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 50 --warmup 5 --exchange unbuffered
step pytest_all 900 python -m pytest tests -m gpu -q -p no:cacheprovider
