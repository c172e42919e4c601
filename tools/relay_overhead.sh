#!/bin/bash
# Host overhead of the relay plane's exchange (two stream synchronisations, one
# allgather, two host barriers) against the stream-ordered peer-write plane: 2 ranks
# on one GPU, tiny grids (the data movement is negligible), one transform per step.
#   tools/relay_overhead.sh <out-dir>
set -o pipefail
out=${1:?out dir}
mkdir -p "$out"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
port=29650
for size in 32 64; do
  for mode in relay peer; do
    if [ $mode = relay ]; then envs="SPFFT_RELAY=force SPFFT_RELAY_VIRTUAL=1"; else envs="SPFFT_RELAY=off"; fi
    port=$((port + 1))
    env $envs OMP_NUM_THREADS=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
      --master-addr=127.0.0.1 --master-port=$port bench.py --gpus 2 --steps 200 --warmup 10 --size $size \
      --transforms 1 > "$out/${mode}_$size.log" 2>&1 || { tail -5 "$out/${mode}_$size.log"; exit 1; }
    grep '^{' "$out/${mode}_$size.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print("'$mode' '$size'", "ms/step", round(d["ms_per_step"],4), "plane", c.get("data_plane"), "stage_ms", c.get("stage_ms"))'
  done
done
