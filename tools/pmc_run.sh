#!/bin/bash
# PMC passes of the stage kernels for one bench.py configuration (one transform
# per step). Every pass is its own rocprofv3 run under a hard time limit; the
# counter sets respect gfx950's per-pass slots (SQ <= 8, TCC <= 4, GRBM <= 2).
#
#   tools/pmc_run.sh <out-dir> <name> <bench.py args...>
#
# Output: <out-dir>/<name>_pmc{A,B}/..._counter_collection.csv and a per-kernel
# table <out-dir>/<name>_pmc.txt (tools/pmc_table.py).
set -o pipefail
out=${1:?out dir}; name=${2:?name}; shift 2
mkdir -p "$out"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
for pass in A B; do
  ctr=${!pass}
  echo "=== $name pass $pass ($(date +%T))"
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$out/${name}_pmc$pass" -o run \
    -- python3 bench.py --steps 3 --warmup 1 --transforms 1 --profile-reps 0 "$@" \
    > "$out/${name}_pmc$pass.log" 2>&1
  rc=$?
  echo "=== rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/${name}_pmc$pass.log"; exit $rc; fi
done
python3 tools/pmc_table.py "$out/${name}_pmcA/run_counter_collection.csv" \
  "$out/${name}_pmcB/run_counter_collection.csv" > "$out/${name}_pmc.txt" 2>&1
cat "$out/${name}_pmc.txt"
