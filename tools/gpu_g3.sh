#!/bin/bash
# rehearsals + Infinity Cache stick hand-off A/B (round 6)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
for mode in "" "--async"; do
  timeout -k 10 200 /opt/conda/bin/mpiexec -n 4 spfft_amd/_native/spfft_bench -d 128 128 128 -r 50 -m 1 -e all \
    -p gpu-gpu --cutoff 0.5 -o "" $mode > gpurun_out/sb4$mode.log 2>&1 || { tail -20 gpurun_out/sb4$mode.log; exit 1; }
  echo "spfft_bench 4 ranks 128^3 $mode: $(grep transforms/s gpurun_out/sb4$mode.log | tr -s ' ' | tr '\n' ';')"
done
bash tools/rehearse4.sh gpurun_out/rehearse > gpurun_out/rehearse.log 2>&1
rc=$?; cut -c1-600 gpurun_out/rehearse.log; [ $rc -ne 0 ] && exit $rc
AB_CONFIGS="t1:--transforms=1 t4:--transforms=4 f32t1:--transforms=1,--precision=single" timeout -k 10 900 bash tools/env_ab.sh gpurun_out/mall s0=SPFFT_EXP_STICK=0 s1=SPFFT_EXP_STICK=1 s2=SPFFT_EXP_STICK=2 s3=SPFFT_EXP_STICK=3 > gpurun_out/mall.log 2>&1
rc=$?; cat gpurun_out/mall.log; for f in gpurun_out/mall/split_*_1.txt; do echo "== $f"; grep "y_\|z_\|sum" $f; done; exit $rc
