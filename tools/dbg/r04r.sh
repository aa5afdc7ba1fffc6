#!/bin/bash
# Round 4: what slows bench.py's host_stream leg (tools/dbg/hs_probe.py).
set -e
mkdir -p gpurun_out
for m in none_stream batch_stream none; do
  timeout -k 10 200 python3 tools/dbg/hs_probe.py $m >> gpurun_out/r04r_hs_probe2.txt 2>&1
done
