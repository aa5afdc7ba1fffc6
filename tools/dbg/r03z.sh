set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03z_pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03z_smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r03z_bench.json 2> gpurun_out/r03z_bench.err
tail -3 gpurun_out/r03z_pytest_gpu.log; cat gpurun_out/r03z_smoke.log
python -c "import json;d=json.load(open('gpurun_out/r03z_bench.json'));print(d['value'],d['kernel_ms'],d['roofline']['valu'])"
