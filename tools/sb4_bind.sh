#!/bin/bash
# spfft_bench, 4 ranks sharing one GPU at 128^3: default process binding against none.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
out=${1:-gpurun_out/sb4}; mkdir -p "$out"
MPIEXEC=$(command -v mpiexec || echo /opt/conda/bin/mpiexec)
"$MPIEXEC" --version 2>&1 | head -2
for b in default none; do for a in "" "--async"; do
  extra=""; [ $b = none ] && extra="--bind-to none"
  timeout -k 10 200 "$MPIEXEC" $extra -n 4 spfft_amd/_native/spfft_bench -d 128 128 128 -r 50 -m 2 -e all -p gpu-gpu --cutoff 0.5 $a -o "$out/sb4_${b}$a.json" > "$out/sb4_${b}$a.log" 2>&1 || { tail -5 "$out/sb4_${b}$a.log"; exit 1; }
  echo "bind=$b $a: $(grep 'transforms/s' "$out/sb4_${b}$a.log" | tr -s ' ' | tr '\n' ';')"
done; done
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null
