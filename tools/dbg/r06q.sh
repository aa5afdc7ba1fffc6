# Round 6: SSIM matrix-core kernel ablations (trivial epilogue, no plane
# loads, no window staging, skeleton) -- per-kernel times from a kernel trace.
mkdir -p gpurun_out || exit 1
cd /tmp && export TMPDIR=/tmp
for lib in epst nostage skel; do
  L=libme_hip_$lib.so; [ $lib = cur ] && L=libme_hip.so
  ME_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r06q_$lib -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-stream --no-4k --no-single --no-ssd --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r06q_$lib.log 2>&1
  rc=$?; [ $rc -le 1 ] || exit $rc  # 1: the ablation's parity failure, expected
done
