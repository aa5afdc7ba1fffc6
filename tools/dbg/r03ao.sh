set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r03ao_ssd_batch_ab.jsonl
export ME_HIP_LIB=libme_hip_tune.so
timeout -k 10 120 python -u tools/dbg/ssd_batch_ab.py >> $O
ME_MFMA_BATCH=0 timeout -k 10 120 python -u tools/dbg/ssd_batch_ab.py >> $O
AB_CONFIG=4k AB_FRAMES=8 timeout -k 10 120 python -u tools/dbg/ssd_batch_ab.py >> $O
AB_CONFIG=4k AB_FRAMES=8 ME_MFMA_BATCH=0 timeout -k 10 120 python -u tools/dbg/ssd_batch_ab.py >> $O
cat $O
unset ME_HIP_LIB
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03ao_pytest_gpu.log 2>&1
tail -2 gpurun_out/r03ao_pytest_gpu.log
