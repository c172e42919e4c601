set -o pipefail
mkdir -p gpurun_out/r2t8
for T in 4 8 4 8 3; do timeout -k 10 120 python bench.py --transforms $T > gpurun_out/r2t8/t$T.json 2>/dev/null || exit 1; python -c "import json; d=json.load(open('gpurun_out/r2t8/t$T.json')); print('T=$T', round(d['value'],1))"; done
for T in 1 4; do timeout -k 10 120 python bench.py --transforms $T --type r2c > gpurun_out/r2t8/r$T.json 2>/dev/null || exit 1; python -c "import json; d=json.load(open('gpurun_out/r2t8/r$T.json')); print('r2c T=$T', round(d['value'],1))"; done
