set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread -k "band_walk or spans" > gpurun_out/r05b_pytest_mfma.log 2>&1; rc=$?; echo pytest rc=$rc; tail -30 gpurun_out/r05b_pytest_mfma.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05b_pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -30 gpurun_out/r05b_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py --steps 20 --no-cpu --no-stream --no-4k > gpurun_out/r05b_bench.json 2> gpurun_out/r05b_bench.err; echo bench rc=$?
