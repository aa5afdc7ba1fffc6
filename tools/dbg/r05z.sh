set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05z}
timeout -k 10 150 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 100 --timeout-method thread -k "band_walk_segments and auto" > gpurun_out/${T}_pytest0.log 2>&1; rc=$?; echo pytest0 rc=$rc; tail -5 gpurun_out/${T}_pytest0.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_stream.py tests/test_gpu_bench_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/${T}_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 150 python3 tools/ssd_ab.py --frames 1,16 --configs 1080p,4k --tag bw --ms 300 >> gpurun_out/${T}_ab.jsonl 2>> gpurun_out/${T}_ab.err; rc=$?; echo "bw rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
ME_PATH=prepass timeout -k 10 150 python3 tools/ssd_ab.py --frames 1,16 --configs 1080p,4k --tag prepass --ms 300 >> gpurun_out/${T}_ab.jsonl 2>> gpurun_out/${T}_ab.err; rc=$?; echo "prepass rc=$rc"
cat gpurun_out/${T}_ab.jsonl
timeout -k 10 120 python3 tools/bw_stamps.py 1080p 16 > gpurun_out/${T}_bw_stamps.txt 2>&1; rc=$?; cat gpurun_out/${T}_bw_stamps.txt
