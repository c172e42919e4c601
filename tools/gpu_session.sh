set -o pipefail
mkdir -p gpurun_out/${S14_OUT:-r1_s14}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${S14_OUT:-r1_s14}/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${S14_OUT:-r1_s14}/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/${S14_OUT:-r1_s14}/bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${S14_OUT:-r1_s14}/prof -o run -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/${S14_OUT:-r1_s14}/prof.log 2>&1
