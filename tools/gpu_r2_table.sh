#!/bin/bash
# README performance table: one bench.py run per configuration on one box.
set -o pipefail
out=gpurun_out/${1:-r2table}
mkdir -p $out
i=0
while read -r args; do
  i=$((i+1))
  timeout -k 10 150 python bench.py $args > $out/t$i.json 2>/dev/null || { echo "failed: $args"; exit 1; }
  python -c "import json; d=json.load(open('$out/t$i.json')); print('$args'.ljust(60), round(d['value'],1))"
done <<'LIST'
--transforms 1
--transforms 4
--type r2c --transforms 1
--type r2c --transforms 4
--precision single --transforms 1
--precision single --transforms 4
--size 128 --transforms 4
--cutoff 0.25 --transforms 4
--size 512 --type r2c --precision single --transforms 1 --steps 10
--size 512 --transforms 1 --steps 10
--size 240 --transforms 4
--size 200 --transforms 4
--size 180 --transforms 4
--size 100 --transforms 4
--size 64 --transforms 4
LIST
