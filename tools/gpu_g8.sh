#!/bin/bash
# z forward sub-batch A/B at T = 4 (round 6)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
AB_CONFIGS="t4:--transforms=4 f32t4:--transforms=4,--precision=single r512:--size=512,--type=r2c,--precision=single,--transforms=4" timeout -k 10 1100 bash tools/env_ab.sh gpurun_out/zfsub s0=SPFFT_ZF_SUB=0 s2=SPFFT_ZF_SUB=2 s1=SPFFT_ZF_SUB=1 > gpurun_out/zfsub.log 2>&1
rc=$?; cat gpurun_out/zfsub.log; for f in gpurun_out/zfsub/split_*_1.txt; do echo "== $f"; grep "z_forward\|sum" $f; done; exit $rc
