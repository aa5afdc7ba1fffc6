set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05s}
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread -k "not lean and not prepass" > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/${T}_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
for A in 0 1 2; do
  ME_HIP_LIB=libme_hip_tune.so ME_BW_ABL=$A timeout -k 10 100 python3 tools/ssd_ab.py --frames 16 --configs 1080p --tag abl$A --ms 300 >> gpurun_out/${T}_abl.jsonl 2>> gpurun_out/${T}_abl.err; rc=$?; echo "abl $A rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done
for P in prepass auto; do
  ME_PATH=$P timeout -k 10 150 python3 tools/ssd_ab.py --frames 1,16 --configs 1080p,4k --tag $P --ms 300 >> gpurun_out/${T}_abl.jsonl 2>> gpurun_out/${T}_abl.err; rc=$?; echo "path $P rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done
cat gpurun_out/${T}_abl.jsonl
timeout -k 10 120 python3 tools/bw_stamps.py 1080p 16 > gpurun_out/${T}_bw_stamps.txt 2>&1; rc=$?; cat gpurun_out/${T}_bw_stamps.txt
