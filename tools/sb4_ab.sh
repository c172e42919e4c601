#!/bin/bash
# spfft_bench, 4 ranks sharing one GPU at 128^3: the in-tree libraries against the
# libraries in spfft_amd/_native/variants/<name>/ (LD_LIBRARY_PATH overrides the
# binary's RUNPATH), synchronous and --async, two alternated rounds.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
out=${1:-gpurun_out/sb4ab}; shift; mkdir -p "$out"
MPIEXEC=$(command -v mpiexec || echo /opt/conda/bin/mpiexec)
for round in 1 2; do for v in base "$@"; do for a in "" "--async"; do
  if [ "$v" = base ]; then lp=""; else lp="$PWD/spfft_amd/_native/variants/$v"; fi
  LD_LIBRARY_PATH="$lp${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH}" timeout -k 10 200 "$MPIEXEC" -n 4 \
    spfft_amd/_native/spfft_bench -d 128 128 128 -r 50 -m 2 -e all -p gpu-gpu --cutoff 0.5 $a \
    -o "$out/${v}_$round$a.json" > "$out/${v}_$round$a.log" 2>&1 || { tail -5 "$out/${v}_$round$a.log"; exit 1; }
  echo "$v round$round $a: $(grep 'transforms/s' "$out/${v}_$round$a.log" | tr -s ' ' | tr '\n' ';')"
done; done; done
