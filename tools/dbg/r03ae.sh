set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/r03ae_bench.json 2> gpurun_out/r03ae_bench.err
python -c "import json;d=json.load(open('gpurun_out/r03ae_bench.json'));print(d['value'],d['kernel_ms'],d['roofline']['valu'],d['single_frame']['kernel_ms'],d['stripe_4k']['value'])"
FLOW_STAMPS_SAVE=gpurun_out/r03ae_flow_single.npy timeout -k 10 100 python -u tools/flow_stamps.py > gpurun_out/r03ae_flow_stamps.txt 2>&1
FLOW_STAMPS_SAVE=gpurun_out/r03ae_flow_batch8.npy timeout -k 10 100 python -u tools/flow_stamps.py batch8 >> gpurun_out/r03ae_flow_stamps.txt 2>&1
cat gpurun_out/r03ae_flow_stamps.txt | grep -v amdgpu.ids
