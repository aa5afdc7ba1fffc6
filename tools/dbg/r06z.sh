# Round 6: the 8K 8x8 SSD bench line (its roofline's valu figure from the
# committed SQ pass) and __graft_entry__.smoke() on this build.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --config 8k --cost ssd --steps 2 --warmup 1 --no-cpu --no-stream --no-4k --no-single --no-ssim > gpurun_out/r06z_8k_ssd_bench.json 2> gpurun_out/r06z_8k_ssd_bench.err
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06z_smoke.log 2>&1
