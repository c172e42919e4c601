set -o pipefail
out=gpurun_out/r2rt; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for sz in 200 180; do for v in base r1; do L=""; [ $v = r1 ] && L=spfft_amd/_native/variants/libspfft_amd_r1.so
 SPFFT_AMD_LIBRARY=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p_${v}_$sz -o run -- python3 bench.py --size $sz --transforms 1 --steps 20 > $out/p_${v}_$sz.log 2>&1 || exit 1
 echo "== $v $sz $(grep -o '"value": [0-9.]*' $out/p_${v}_$sz.log)"; python tools/kstats.py $out/p_${v}_$sz/run_kernel_stats.csv | head -6 | cut -c1-70,100-
done; done
