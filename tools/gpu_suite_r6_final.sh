cd $GRAFT_REPO_ROOT
bash tools/gpu_suite.sh gpurun_out/suite4 tests smoke bench bench32 > gpurun_out/suite4.log 2>&1 || exit $?
MPIEXEC=$(command -v mpiexec || echo /opt/conda/bin/mpiexec)
for a in "" "--async"; do
  timeout -k 10 200 "$MPIEXEC" -n 4 spfft_amd/_native/spfft_bench -d 128 128 128 -r 50 -m 2 -e all -p gpu-gpu --cutoff 0.5 $a -o gpurun_out/suite4/sb4$a.json > gpurun_out/suite4/sb4$a.log 2>&1 || exit $?
  echo "spfft_bench 4 ranks 128^3 $a: $(grep 'transforms/s' gpurun_out/suite4/sb4$a.log | tr -s ' ' | tr '\n' ';')" >> gpurun_out/suite4.log
done
for ex in compact unbuffered; do
  timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=$((29970 + ${#ex})) bench.py --gpus 2 --steps 100 --warmup 5 --size 256 --exchange $ex > gpurun_out/suite4/b2_$ex.json 2> gpurun_out/suite4/b2_$ex.err || exit $?
  echo "bench 2 ranks 256^3 T=4 $ex: $(tail -1 gpurun_out/suite4/b2_$ex.json | cut -c1-160)" >> gpurun_out/suite4.log
done
