#!/bin/bash
# A/B of the wide 512-thread shapes on the configurations they affect (with --check).
set -o pipefail
out=gpurun_out/${1:-r2wide}
mkdir -p $out
lib() { [ "$1" = base ] && echo "" || echo "spfft_amd/_native/variants/libspfft_amd_$1.so"; }
run() {  # variant, tag, args
  SPFFT_AMD_LIBRARY=$(lib $1) timeout -k 10 180 python bench.py --transforms 1 --steps 10 $3 > $out/$1_$2.json 2>/dev/null || { echo "$1 $2 failed"; exit 1; }
  python -c "import json; d=json.load(open('$out/$1_$2.json')); print('$1 $2', round(d['value'],1), d['config']['check_error'])"
}
for r in 1 2; do
  for v in base wf512; do run $v r2c512f "--size 512 --type r2c --precision single $( [ $r = 1 ] && echo --check)"; done
  for v in base wd512; do run $v c2c512d "--size 512 $( [ $r = 1 ] && echo --check)"; done
  for v in base wf256; do run $v c2c256f "--precision single $( [ $r = 1 ] && echo --check)"; done
  for v in base wf256; do run $v r2c512f2 "--size 512 --type r2c --precision single"; done
done
