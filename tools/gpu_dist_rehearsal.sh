# Rehearse the driver's multi-rank bench launch on a 1-GPU box (ranks share the
# device; the library moves exchange data by IPC peer writes).
set -o pipefail
out=gpurun_out/r1_s14_dist; mkdir -p $out
for np in 2 4; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np \
    --master-addr 127.0.0.1 --master-port $((29500+np)) bench.py --gpus $np --steps 10 --warmup 3 --check \
    > $out/bench_np$np.log 2>&1 || exit $?
done
timeout -k 10 240 python bench.py --steps 50 --warmup 5 --check > $out/bench_np1_check.log 2>&1
