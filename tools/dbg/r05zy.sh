set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zy}; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullframe.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
C="--no-cpu --no-stream --no-4k --no-single --no-ssim --no-ssd --config 8k --steps 3 --warmup 1"
for V in libme_hip.so libme_hip_v_old.so libme_hip.so libme_hip_v_old.so; do
  ME_HIP_LIB=$V timeout -k 10 200 python3 bench.py $C > gpurun_out/${T}_$V.json 2> gpurun_out/${T}_$V.err; rc=$?; echo "$V bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_$V.json')); print('$V', round(d['ms_per_step'],3), d['roofline'].get('valu',{}).get('frac'), d['parity'])" | tee -a gpurun_out/${T}_ab.txt
done
