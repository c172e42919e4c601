#!/bin/bash
# Parametrised GPU-box runner (replaces the round-1/2 one-off session scripts).
#
#   tools/gpu_suite.sh <out-dir> <suite> [<suite> ...]
#
# Suites:
#   tests          full `pytest -m gpu` suite
#   tests:<expr>   `pytest -m gpu -k <expr>`
#   smoke          __graft_entry__.smoke()
#   bench          headline bench.py (T=4) and --transforms 1
#   bench32        256^3 C2C fp32 and 512^3 R2C fp32 (BASELINE config 5 shape) bench lines
#   prof           rocprofv3 --kernel-trace --stats of the headline bench (T=1 and T=4)
#   prof32         the same for the fp32 configurations
#   rccl           the RCCL data plane: RCCL self-loopback GPU tests and the
#                  2-rank shared-device RCCL probe (outcome recorded either way)
#   cmd:<shell>    any other command (one step)
#
# Every GPU step runs under its own time limit; the runner stops at the first
# crash, abort or timeout (exit >= 124, 134, 139) and never retries a step.
set -o pipefail
out=${1:?out dir}; shift
mkdir -p "$out"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1

step() {
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 6 "$out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "stopping after $name (rc=$rc)"; exit $rc
  fi
  return 0
}

prof() {  # prof <name> <bench args...>
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}" &&
   step "prof_$name" 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$out/prof_$name" -o run -- python3 bench.py "$@") || exit $?
  python3 tools/kstats.py "$out/prof_$name/run_kernel_stats.csv" > "$out/kstats_$name.txt" 2>&1
  head -n 12 "$out/kstats_$name.txt"
}

PYT="python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread"
ncmd=0
for s in "$@"; do
  case "$s" in
    tests) step gpu_tests 1000 $PYT tests -m gpu -q ;;
    tests:*) step gpu_tests_k 600 $PYT tests -m gpu -q -k "${s#tests:}" ;;
    smoke) step smoke 180 python __graft_entry__.py smoke ;;
    bench)
      step bench_t4 300 python bench.py --steps 200 --warmup 10
      step bench_t1 300 python bench.py --steps 200 --warmup 10 --transforms 1 ;;
    bench32)
      step bench_c2c256_f32_t1 300 python bench.py --steps 200 --warmup 10 --precision single --transforms 1
      step bench_c2c256_f32 300 python bench.py --steps 200 --warmup 10 --precision single
      step bench_r2c512_f32 300 python bench.py --steps 50 --warmup 5 --precision single --type r2c --size 512 ;;
    prof)
      prof t1 --steps 20 --transforms 1
      prof t4 --steps 20 ;;
    prof32)
      prof f32_t1 --steps 20 --transforms 1 --precision single
      prof r2c512_f32 --steps 10 --precision single --type r2c --size 512 ;;
    rccl)
      step rccl_tests 600 $PYT tests -m gpu -q -k "rccl"
      SPFFT_GPU_EXCHANGE=rccl NCCL_DEBUG=WARN step rccl_shared_device 180 \
        python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
        --master-port=29561 tools/rccl_probe.py COMPACT_BUFFERED --iters=2 ;;
    ab:*)
      # ab:<v1>,<v2>,...: kernel stats of the headline fp64, 256^3 fp32 and 512^3 R2C
      # fp32 problems (one transform per step) for the main library ("main") and the
      # variants built by tools/build_variants.py
      IFS=, read -r -a vs <<< "${s#ab:}"
      for v in "${vs[@]}"; do
        if [ "$v" = main ]; then unset SPFFT_AMD_LIBRARY; else
          export SPFFT_AMD_LIBRARY=$PWD/spfft_amd/_native/variants/libspfft_amd_$v.so; fi
        prof "${v}_f64" --steps 20 --warmup 5 --transforms 1
        prof "${v}_f32" --steps 20 --warmup 5 --transforms 1 --precision single
        prof "${v}_r2c512" --steps 10 --warmup 3 --transforms 1 --precision single --type r2c --size 512
      done
      unset SPFFT_AMD_LIBRARY ;;
    cmd:*) ncmd=$((ncmd + 1)); step cmd$ncmd 900 bash -c "${s#cmd:}" ;;
    *) echo "unknown suite $s"; exit 2 ;;
  esac
done
