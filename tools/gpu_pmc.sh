#!/bin/bash
source tools/gpu_run.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step pmc1 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc1 -o run --output-format csv -- python bench.py --steps 2 --warmup 1
step pmc2 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc2 -o run --output-format csv -- python bench.py --steps 2 --warmup 1
step pmc3 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc3 -o run --output-format csv -- python bench.py --steps 2 --warmup 1
step pmc4 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc4 -o run --output-format csv -- python bench.py --steps 2 --warmup 1
