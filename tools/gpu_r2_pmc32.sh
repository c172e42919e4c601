#!/bin/bash
# PMC passes comparing the fp32 and fp64 stage kernels (256^3 C2C, one transform per step).
source tools/gpu_run.sh
tag=${1:-r2pmc32}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for prec in single double; do
  step ${tag}_${prec}_A 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/$tag/${prec}_A -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --transforms 1 --precision $prec
  step ${tag}_${prec}_B 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM --kernel-trace -d gpurun_out/$tag/${prec}_B -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --transforms 1 --precision $prec
  python3 tools/pmc_summary.py $(find gpurun_out/$tag/${prec}_* -name "*counter_collection.csv") > gpurun_out/$tag/summary_$prec.txt
done
cat gpurun_out/$tag/summary_single.txt | head -60
