set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullframe.py tests/test_gpu_parity.py tests/test_gpu_mfma.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03t_parity.log 2>&1
bash tools/profile.sh r03t_8k_ssd --steps 3 --warmup 1 --no-cpu --no-stream --no-4k --cost ssd --config 8k > gpurun_out/r03t_prof.txt 2>&1
