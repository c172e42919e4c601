#!/bin/bash
# Session 5: in-process peer-write fix + PMC counters of the current stage kernels.
source tools/gpu_run.sh
step pytest_vr 600 python -m pytest tests/test_gpu_transform.py -m gpu -q -p no:cacheprovider -x -k "virtual or multi"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python bench.py --steps 3 --warmup 1"
step pmcA 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmcA -o run --output-format csv -- $B
step pmcB 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM --kernel-trace -d gpurun_out/pmcB -o run --output-format csv -- $B
step pmcC 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/pmcC -o run --output-format csv -- $B
step pmcD 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcD -o run --output-format csv -- $B
step pmcE 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcE -o run --output-format csv -- $B
step pmcF 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-trace -d gpurun_out/pmcF -o run --output-format csv -- $B
