set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zb}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; tail -5 gpurun_out/${T}_pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
for P in auto lean prepass; do
  ME_PATH=$P timeout -k 10 150 python3 tools/ssd_ab.py --frames 1,16 --configs 1080p,4k --tag $P --ms 300 >> gpurun_out/${T}_ab.jsonl 2>> gpurun_out/${T}_ab.err; rc=$?; echo "$P rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done
cat gpurun_out/${T}_ab.jsonl
