#!/bin/bash
# Full GPU suite with the mixed-radix sizes, then a size sweep: FftMR vs the run-time engine.
set -o pipefail
out=gpurun_out/mrsweep
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -n 40 $out/pytest.log; exit 1; }
tail -n 2 $out/pytest.log
V=spfft_amd/_native/variants/libspfft_amd_nomr.so
for p in double single; do
  for n in 96 120 144 160 180 216 288 320 360 384 400 480; do
    s=20; [ $n -ge 320 ] && s=8
    line="$n $p:"
    for v in base nomr; do
      lib=""; [ $v = nomr ] && lib=$V
      SPFFT_AMD_LIBRARY=$lib timeout -k 10 180 python bench.py --size $n --precision $p --transforms 1 --steps $s --warmup 2 > $out/b.json 2>$out/b.err || { cat $out/b.err | tail -5; exit 1; }
      line="$line $v=$(python -c "import json; print(round(json.load(open('$out/b.json'))['value']))")"
    done
    echo "$line"
  done
done
