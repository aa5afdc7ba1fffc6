set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zz3}; export TMPDIR=/tmp
for R in 1 2; do
for E in "X=0" "ME_STREAM_BATCH=8" "ME_STREAM_BATCH=12" "ME_STREAM_BATCH=16" "ME_STREAM_BATCH=16 ME_STREAM_AHEAD=3" "ME_STREAM_BATCH=24"; do
  echo "== $E" >> gpurun_out/${T}.txt
  env ME_HIP_LIB=libme_hip_tune.so $E timeout -k 10 120 python3 tools/dbg/stream_trace.py 64 >> gpurun_out/${T}.txt 2>&1 || exit $?
done; done
grep -v amdgpu gpurun_out/${T}.txt
