set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zm}; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/${T}_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
C="--no-cpu --no-stream --no-4k --no-single --no-ssim"
bash tools/profile.sh ${T}_8k_ssd --steps 2 --warmup 1 $C --cost ssd --config 8k > gpurun_out/${T}_prof6.txt 2>&1; echo prof6 rc=$?
bash tools/profile.sh ${T}_4k_ssd_prepass --steps 4 --warmup 1 $C --cost ssd --config 4k > gpurun_out/${T}_prof5.txt 2>&1; echo prof5 rc=$?
