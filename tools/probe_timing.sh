cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/cmp3; p=29900
for probe in none relay; do p=$((p+1))
  if [ "$probe" = none ]; then pa="--planes-probe 0"; else pa="--planes-probe 1 --probe-planes $probe"; fi
  timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=$p bench.py --gpus 2 --steps 50 --warmup 5 --size 256 --exchange compact --transforms 1 --profile-reps 0 --plane ipc --timing $pa > gpurun_out/cmp3/$probe.json 2> gpurun_out/cmp3/$probe.err || { tail -5 gpurun_out/cmp3/$probe.err; exit 1; }
done
