set -o pipefail
out=gpurun_out/r2big2; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base w1024; do L=""; [ $v != base ] && L=spfft_amd/_native/variants/libspfft_amd_$v.so
  SPFFT_AMD_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p_$v -o run -- python3 bench.py --size 1024 --transforms 1 --steps 3 --warmup 1 --check > $out/p_$v.log 2>&1 || { tail $out/p_$v.log; exit 1; }
  echo "== $v $(grep -o '"value": [0-9.]*' $out/p_$v.log) $(grep -o '"roundtrip": [0-9.e-]*' $out/p_$v.log)"; python tools/kstats.py $out/p_$v/run_kernel_stats.csv | head -6 | cut -c1-60,100-
done
