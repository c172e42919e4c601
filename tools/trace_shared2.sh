#!/bin/bash
# 2 ranks of bench.py (256^3, T = 1, default plane) sharing the GPU, each under
# rocprofv3 --kernel-trace; per-rank kernel timelines.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
out=${1:-gpurun_out/trace2}
rm -rf "$out"; mkdir -p "$out"
pids=()
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=29691 \
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$out/r$r" -o run -- \
    python3 bench.py --gpus 2 --steps 20 --warmup 3 --transforms 1 --profile-reps 0 --planes-probe 0 \
    > "$out/r$r.log" 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
[ $rc -ne 0 ] && { tail -20 "$out/r0.log" "$out/r1.log"; exit $rc; }
grep '^{' "$out/r0.log" | cut -c1-200
for r in 0 1; do
  f=$(find "$out/r$r" -name '*kernel_trace.csv' | head -1)
  echo "== rank $r"; python3 tools/ktimeline.py "$f" --skip 100 --tail 16
done
