set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=r05zz7
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
for R in 1 2; do for E in "ME_STREAM_HOSTWAIT=0" "X=0"; do
  echo "== $E" >> gpurun_out/${T}.txt
  env ME_HIP_LIB=libme_hip_tune.so $E timeout -k 10 120 python3 tools/dbg/stream_trace.py 64 >> gpurun_out/${T}.txt 2>&1 || exit $?
done; done
echo "== product lib" >> gpurun_out/${T}.txt
timeout -k 10 120 python3 tools/dbg/stream_trace.py 64 >> gpurun_out/${T}.txt 2>&1 || exit $?
grep -v amdgpu gpurun_out/${T}.txt
