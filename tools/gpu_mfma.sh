#!/bin/bash
# MFMA vs VALU DFT-16 throughput probe + VALU/MFMA counters of the probe and of
# the headline stage kernels.
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step mfma_dft 120 ./spfft_amd/_native/mfma_dft
P="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
step pmc_probe 90 timeout -s KILL 60 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc_probe -o run -- ./spfft_amd/_native/mfma_dft
step pmc_bench 120 timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc_bench -o run -- python bench.py --steps 3 --warmup 1
cat gpurun_out/mfma_dft.log
true
