set -o pipefail
out=gpurun_out/r2rt2; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { # name lib env
  env $3 SPFFT_AMD_LIBRARY=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p_$1 -o run -- python3 bench.py --size 200 --transforms 1 --steps 20 > $out/p_$1.log 2>&1 || exit 1
  echo "== $1 $(grep -o '"value": [0-9.]*' $out/p_$1.log)"; python tools/kstats.py $out/p_$1/run_kernel_stats.csv | grep y_ | cut -c1-70,100-
}
run base "" "X=1"
run nodesc "" "SPFFT_COL_DESC=0"
run yslow spfft_amd/_native/variants/libspfft_amd_yslow.so "X=1"
run yslow_nodesc spfft_amd/_native/variants/libspfft_amd_yslow.so "SPFFT_COL_DESC=0"
