set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zq}; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_fullframe.py -x -q --timeout 200 --timeout-method thread -k "mfma8 or 8k_b8_s128_ssd" > gpurun_out/${T}_pytest0.log 2>&1; rc=$?; echo pytest0 rc=$rc; tail -3 gpurun_out/${T}_pytest0.log
[ $rc -eq 0 ] || exit $rc
C="--no-cpu --no-stream --no-4k --no-single --no-ssim --cost ssd --config 8k --steps 4 --warmup 1"
for V in libme_hip.so libme_hip_v_bar.so libme_hip_v_old.so libme_hip.so libme_hip_v_bar.so libme_hip_v_old.so; do
  ME_HIP_LIB=$V timeout -k 10 200 python3 bench.py $C > gpurun_out/${T}_$V.json 2> gpurun_out/${T}_$V.err; rc=$?; echo "$V bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${T}_$V.json')); print('$V', d['ms_per_step'], d.get('kernel_ms'), d['parity'] if 'parity' in d else '')"
done
