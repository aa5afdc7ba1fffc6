set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03al_pytest_gpu.log 2>&1
tail -2 gpurun_out/r03al_pytest_gpu.log
bash tools/profile_all.sh r03al
