set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zg}
timeout -k 10 200 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 150 --timeout-method thread -k "band_walk" > gpurun_out/${T}_pytest0.log 2>&1; rc=$?; echo pytest0 rc=$rc; tail -3 gpurun_out/${T}_pytest0.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_bench_batch.py tests/test_gpu_fullframe.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/${T}_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
for X in 1 0; do
  ME_BW_XT=$X timeout -k 10 150 python3 tools/ssd_ab.py --frames 16 --configs 1080p,4k --tag xt$X --ms 300 >> gpurun_out/${T}_ab.jsonl 2>> gpurun_out/${T}_ab.err; rc=$?; echo "xt$X rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done
ME_PATH=prepass timeout -k 10 150 python3 tools/ssd_ab.py --frames 16 --configs 1080p,4k --tag prepass --ms 300 >> gpurun_out/${T}_ab.jsonl 2>> gpurun_out/${T}_ab.err; rc=$?; echo "prepass rc=$rc"
cat gpurun_out/${T}_ab.jsonl
