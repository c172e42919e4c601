set -o pipefail
o=gpurun_out/${ZEXP_OUT:-r1_s14_zreg}; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "not torch_dist" > $o/pytest.log 2>&1 && \
timeout -k 10 200 python bench.py --check > $o/bench.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 100 > $o/bench2.log 2>&1 && \
timeout -k 10 200 python bench.py --type r2c > $o/bench_r2c.log 2>&1 && \
timeout -k 10 200 python bench.py --precision single > $o/bench_fp32.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 20 --warmup 3 > $o/prof.log 2>&1
