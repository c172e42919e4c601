cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && \
AB_CONFIGS="t4:--transforms=4 t1:--transforms=1" timeout -k 10 900 bash tools/env_ab.sh gpurun_out/zb base=SPFFT_EXP_ZB=0 nt=SPFFT_EXP_ZB=1 ilv=SPFFT_EXP_ZB=2 both=SPFFT_EXP_ZB=3 > gpurun_out/zb.log 2>&1; rc=$?; cat gpurun_out/zb.log; for f in gpurun_out/zb/split_*_1.txt; do echo "== $f"; grep z_backward $f; done; exit $rc
