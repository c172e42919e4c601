#!/bin/bash
# Round 2 PMC passes over the headline bench (each pass its own run, within the per-block limits).
source tools/gpu_run.sh
tag=${1:-r2pmc}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { local n=$1; shift; step ${tag}_$n 120 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/$tag/$n -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1; }
run A TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_LATENCY_sum
run B TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum
run C TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum
run D TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_BUSY_sum
run E SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
python3 tools/pmc_summary.py $(find gpurun_out/$tag -name "*counter_collection.csv") > gpurun_out/$tag/summary.txt
cat gpurun_out/$tag/summary.txt
