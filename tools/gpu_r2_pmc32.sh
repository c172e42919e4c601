#!/bin/bash
# Instruction mix and stalls, fp32 vs fp64 (256^3 C2C, one transform per step).
source tools/gpu_run.sh
tag=pmc32b
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { local n=$1 p=$2; shift 2; step ${tag}_$n 120 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/$tag/$n -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --transforms 1 --precision $p; }
for p in single double; do
  run I$p $p SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
  run S$p $p SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY GRBM_GUI_ACTIVE
done
for p in single double; do
  echo "== $p"
  python3 tools/pmc_summary.py $(find gpurun_out/$tag/I$p gpurun_out/$tag/S$p -name "*counter_collection.csv") | tee gpurun_out/$tag/summary_$p.txt
done
