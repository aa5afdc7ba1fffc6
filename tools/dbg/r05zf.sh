set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zf}
timeout -k 10 150 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 100 --timeout-method thread -k "band_walk_segments" > gpurun_out/${T}_pytest0.log 2>&1; rc=$?; echo pytest0 rc=$rc; tail -3 gpurun_out/${T}_pytest0.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_bench_batch.py tests/test_gpu_fullframe.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/${T}_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
for P in auto prepass; do
  ME_PATH=$P timeout -k 10 150 python3 tools/ssd_ab.py --frames 1,16 --configs 1080p,4k --tag $P --ms 300 >> gpurun_out/${T}_ab.jsonl 2>> gpurun_out/${T}_ab.err; rc=$?; echo "$P rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done
cat gpurun_out/${T}_ab.jsonl
C="--no-cpu --no-stream --no-4k --no-single --no-ssim"
C="--no-cpu --no-stream --no-4k --no-single --no-ssim"
bash tools/profile.sh ${T}_1080p_ssd --steps 20 --warmup 3 $C --cost ssd > gpurun_out/${T}_prof2.txt 2>&1; echo prof2 rc=$?
