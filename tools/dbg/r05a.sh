set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05a_pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -15 gpurun_out/r05a_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
tools/dbg/stream_probe.sh r05a; rc=$?; echo probe rc=$rc; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python bench.py --steps 20 > gpurun_out/r05a_bench.json 2> gpurun_out/r05a_bench.err; echo bench rc=$?
