#!/bin/bash
# GPU transform tests + bench lines after the cache hand-off (round 6)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/g4
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_transform.py tests/test_fuzz.py > gpurun_out/g4/tests.log 2>&1
rc=$?; tail -3 gpurun_out/g4/tests.log; [ $rc -ne 0 ] && { grep -m5 -A20 "FAILED\|Error" gpurun_out/g4/tests.log | head -60; exit $rc; }
for args in "--transforms 1" "--transforms 4" "--transforms 1 --precision single" "--transforms 4 --precision single" "--size 512 --type r2c --precision single --transforms 1" "--size 512 --type r2c --precision single --transforms 4"; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 $args > gpurun_out/g4/b.json 2>/dev/null || exit 1
  echo "$args: $(python3 -c 'import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(r["value"],1), r["config"]["check_error"]["ok"])' gpurun_out/g4/b.json)"
done
