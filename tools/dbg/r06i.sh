# Round 6: full GPU suite and the default bench line (per-leg wall times, the
# new ssd_single_frame leg).
set -e
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06i_pytest_gpu.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r06i_bench.json 2> gpurun_out/r06i_bench.err
