#!/bin/bash
# Session 3 end-of-work validation: full GPU suite, smoke, headline bench (3 runs),
# single-transform bench, reference CLI with -m 4, kernel stats of the headline bench.
source tools/gpu_run.sh
out=gpurun_out/s3final
mkdir -p $out
step gpu_tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 180 python __graft_entry__.py smoke
for r in 1 2 3; do step bench$r 300 python bench.py --steps 200 --warmup 10; done
step bench_t1 300 python bench.py --steps 200 --warmup 10 --transforms 1
step cli64 300 ./spfft_amd/_native/spfft_bench -d 64 64 64 -r 200 -m 4 -o $out/cli64.json -e compact -p gpu-gpu --cutoff 0.5
step cli256 300 ./spfft_amd/_native/spfft_bench -d 256 256 256 -r 30 -m 4 -o $out/cli256.json -e compact -p gpu-gpu --cutoff 0.5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --steps 20
python tools/kstats.py $out/prof/run_kernel_stats.csv > $out/kstats.txt 2>&1
cat $out/kstats.txt
