#!/bin/bash
# PMC comparison of the run-time engine (240^3) and the compile-time engine (256^3).
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
for n in 240 256; do
  step pa_$n 120 timeout -s KILL 90 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d gpurun_out/pa_$n -o run -- python bench.py --steps 2 --warmup 1 --size $n
  step pb_$n 120 timeout -s KILL 90 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d gpurun_out/pb_$n -o run -- python bench.py --steps 2 --warmup 1 --size $n
done
true
