set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for R in 1 2; do for E in "X=0" "ME_STREAM_NOWAIT=1"; do
  echo "== $E" >> gpurun_out/r05zz6.txt
  env ME_HIP_LIB=libme_hip_tune.so $E timeout -k 10 120 python3 tools/dbg/stream_trace.py 64 >> gpurun_out/r05zz6.txt 2>&1 || exit $?
done; done
ME_HIP_LIB=libme_hip_tune.so ME_STREAM_NOWAIT=1 ME_STREAM_TIMING=1 timeout -k 10 120 python3 tools/dbg/stream_trace.py 64 2>&1 | tail -14 >> gpurun_out/r05zz6.txt
grep -v amdgpu gpurun_out/r05zz6.txt
