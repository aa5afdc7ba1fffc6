# Final checks of the round on the current build: GPU suite, smoke(), default bench line
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03bf_pytest_gpu.log 2>&1
tail -2 gpurun_out/r03bf_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03bf_smoke.log 2>&1
cat gpurun_out/r03bf_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r03bf_bench.json 2> gpurun_out/r03bf_bench.err
cat gpurun_out/r03bf_bench.json
