cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g1 && \
timeout -k 10 200 /opt/conda/bin/mpiexec -n 4 spfft_amd/_native/spfft_bench -d 128 128 128 -r 50 -m 1 -e all -p gpu-gpu --cutoff 0.5 -o gpurun_out/g1/sb4.json > gpurun_out/g1/sb4.log 2>&1 && grep transforms/s gpurun_out/g1/sb4.log && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_torch_dist.py > gpurun_out/g1/tdist.log 2>&1; rc=$?; tail -50 gpurun_out/g1/tdist.log; exit $rc
