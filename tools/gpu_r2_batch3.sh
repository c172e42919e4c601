#!/bin/bash
# Host-side cost of batched vs unbatched multi-transform calls (timing tree, 64^3, T=4).
source tools/gpu_run.sh
out=gpurun_out/batch3
mkdir -p $out
for b in 0 1; do
  SPFFT_BATCH=$b timeout -k 10 120 python bench.py --size 64 --transforms 4 --steps 400 --warmup 5 --timing > $out/t$b.json 2> $out/t$b.err || exit 1
  cat $out/t$b.json | cut -c1-120
  grep -v "amdgpu.ids" $out/t$b.err | head -40
done
