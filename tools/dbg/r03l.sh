set -e
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/dbg/alloc_probe.py > gpurun_out/r03l_alloc.json 2>/dev/null
timeout -k 10 150 python -u tools/dbg/alloc_probe.py >> gpurun_out/r03l_alloc.json 2>/dev/null
