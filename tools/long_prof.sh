#!/bin/bash
# Kernel stats of the long-line path (four-step / Bluestein in global memory)
# against in-LDS lines of similar length: tools/long_prof.sh <out-dir>
set -o pipefail
out=${1:?out dir}
mkdir -p "$out"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
for case in "64,64,4096 double" "64,64,6144 double" "64,64,8192 double" "4096,64,64 double" \
            "6144,64,64 double" "8192,64,64 double" "64,64,8192 single" "8192,64,64 single"; do
  set -- $case
  name="$(echo $1 | tr , x)_$2"
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$name" -o run \
    -- python3 tools/long_bench.py --dims "$1" --precision "$2" --steps 10 > "$out/$name.log" 2>&1
  rc=$?
  tail -1 "$out/$name.log"
  [ $rc -ne 0 ] && exit $rc
  python3 tools/kstats.py "$out/$name/run_kernel_stats.csv" > "$out/kstats_$name.txt" 2>&1
done
exit 0
