set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zh}
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 200 --timeout-method thread -k "mfma8" > gpurun_out/${T}_pytest0.log 2>&1; rc=$?; echo pytest0 rc=$rc; tail -3 gpurun_out/${T}_pytest0.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_fullframe.py tests/test_gpu_parity.py tests/test_gpu_bench_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/${T}_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
C="--no-cpu --no-stream --no-4k --no-single --no-ssim"
SIZED=1 bash tools/profile.sh ${T}_8k_ssd --steps 2 --warmup 1 $C --cost ssd --config 8k > gpurun_out/${T}_prof6.txt 2>&1; echo prof6 rc=$?
