set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05u}
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 300 --timeout-method thread -k "not lean and not prepass" > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/${T}_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
for W in 1 2; do
  ME_HIP_LIB=libme_hip_tune.so ME_BW_WG=$W timeout -k 10 150 python3 tools/ssd_ab.py --frames 1,16 --configs 1080p,4k --tag wg$W --ms 300 >> gpurun_out/${T}_ab.jsonl 2>> gpurun_out/${T}_ab.err; rc=$?; echo "wg $W rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done
ME_PATH=prepass timeout -k 10 150 python3 tools/ssd_ab.py --frames 1,16 --configs 1080p,4k --tag prepass --ms 300 >> gpurun_out/${T}_ab.jsonl 2>> gpurun_out/${T}_ab.err; rc=$?; echo "prepass rc=$rc"
cat gpurun_out/${T}_ab.jsonl
