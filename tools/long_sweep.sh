#!/bin/bash
# Long-line path rates (tools/long_bench.py) for the round-4 shapes, one line each.
out=${1:-gpurun_out/long}
mkdir -p "$out"
: > "$out/long_bench_lines.txt"
for spec in "4096,64,64 double" "6144,64,64 double" "64,64,4096 double" "64,64,6144 double" \
            "64,64,8192 double" "64,64,8192 single" "8192,64,64 double" "8192,64,64 single"; do
  set -- $spec
  timeout -k 10 120 python tools/long_bench.py --dims "$1" --precision "$2" >> "$out/long_bench_lines.txt" 2>&1 || exit 1
done
cat "$out/long_bench_lines.txt"
