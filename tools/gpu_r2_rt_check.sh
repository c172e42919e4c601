set -o pipefail
out=gpurun_out/r2rt3; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $out/pytest.log 2>&1; tail -n 2 $out/pytest.log
for args in "--size 200 --transforms 1" "--size 180 --transforms 1" "--size 240 --transforms 1" "--transforms 1" "--size 200" "--size 240"; do
  timeout -k 10 120 python bench.py $args 2>/dev/null | python -c "import json,sys; print('$args'.ljust(30), round(json.load(sys.stdin)['value'],1))" || exit 1
done
