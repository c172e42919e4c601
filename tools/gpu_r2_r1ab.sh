set -o pipefail
# round-1 library vs current on one box, --transforms 1, interleaved
for args in "--precision single" "--type r2c" "--size 128" "--size 100" "--cutoff 0.25" "--size 512 --type r2c --precision single --steps 10" "--size 64" "--type r2c --precision single"; do
 for v in base r1; do L=""; [ $v = r1 ] && L=spfft_amd/_native/variants/libspfft_amd_r1.so
  SPFFT_AMD_LIBRARY=$L timeout -k 10 120 python bench.py --transforms 1 $args 2>/dev/null | python -c "import json,sys; print('$v'.ljust(5), '$args'.ljust(50), round(json.load(sys.stdin)['value'],1))" || exit 1
 done
done
