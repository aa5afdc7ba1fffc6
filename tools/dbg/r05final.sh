set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05f}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/${T}_pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1; echo smoke rc=$?
bash tools/profile_all.sh $T; echo profile rc=$?
