set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py -x -q --timeout 200 --timeout-method thread > gpurun_out/mfma_tests.log 2>&1; rc=$?; tail -3 gpurun_out/mfma_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in 1080p 4k; do for bm in 1 0; do
 ME_HIP_LIB=libme_hip_tune.so ME_MFMA_BM=$bm timeout -k 10 120 python bench.py --cost ssd --config $cfg --no-cpu --no-stream --steps 20 --warmup 3 > gpurun_out/b_${cfg}_$bm.json || exit 1
 python3 -c "import json;d=json.load(open('gpurun_out/b_${cfg}_$bm.json'));print('$cfg bm=$bm', round(d['ms_per_step'],4), d['kernel_ms'], '%.3g'%d['value'])"
done; done
