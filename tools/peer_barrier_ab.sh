#!/bin/bash
# A/B of the peer-plane barrier modes (SPFFT_PEER_BARRIER): bench.py UNBUFFERED on
# 2 ranks sharing the GPU. Output: gpurun_out/<dir>/bench_<mode>_<size>_t<T>.json
out=${1:-gpurun_out/barrier_ab}
mkdir -p "$out"
port=29571
for size in 128 256; do
  for T in 1 4; do
    for mode in stream channel host; do
      port=$((port + 1))
      SPFFT_PEER_BARRIER=$mode timeout -k 10 120 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=$port bench.py --gpus 2 \
        --steps 20 --warmup 3 --size $size --exchange unbuffered --transforms $T \
        > "$out/bench_${mode}_${size}_t${T}.json" 2> "$out/bench_${mode}_${size}_t${T}.err" || exit 1
      echo "$mode $size T=$T done"
    done
  done
done
