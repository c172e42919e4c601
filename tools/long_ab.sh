#!/bin/bash
# Same-box A/B of library builds on the long-line (four-step) path: long_bench.py
# rates and per-kernel stats, each library (name=path; base = in-tree) alternated twice.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
out=${1:?out}; shift; mkdir -p "$out"
export TMPDIR=/tmp
for round in 1 2; do for setting in base "$@"; do
  name=${setting%%=*}; lib=${setting#*=}
  if [ "$name" = base ]; then unset SPFFT_AMD_LIBRARY; else export SPFFT_AMD_LIBRARY=$lib; fi
  for case in ${CASES:-"8192,64,64 double" "4096,64,64 double" "64,64,8192 double" "8192,64,64 single"}; do
    set -- $case
    c="$(echo $1 | tr , x)_$2"; d="$out/${name}_${c}_$round"
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run \
      -- python3 tools/long_bench.py --dims "$1" --precision "$2" --steps 10 > "$d.log" 2>&1 || { tail -3 "$d.log"; exit 1; }
    python3 tools/kstats.py "$d/run_kernel_stats.csv" > "$d.kstats" 2>&1
    echo "$name round$round $c: $(tail -1 "$d.log") | $(grep -E '^void long_' "$d.kstats" | sed -E 's/void (long_[a-z]+)_kernel<CtEng<[a-z]+, ([0-9]+), (-?1).*avg_us= *([0-9.]+).*/\1 \2 \3 \4/' | tr '\n' ';')"
  done
done; done
unset SPFFT_AMD_LIBRARY
