#!/bin/bash
# Round 4: item-kernel per-item scalar divisions and the rows-only epilogue --
# GPU suite, then 4K / 8K SAD batch times against the previous build
# (libme_hip_old.so), interleaved twice; the pair-record stream A/B.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04t_pytest_gpu.log 2>&1
OUT=gpurun_out/r04t_ab.txt
C="--no-cpu --no-stream --no-4k --no-single --no-ssd"
for rep in 1 2; do
  for lib in libme_hip_old.so libme_hip.so; do
    r4=$(ME_HIP_LIB=$lib timeout -k 10 120 python3 bench.py --config 4k --steps 8 --warmup 2 $C | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['kernel_ms'],3), d['parity'])")
    r8=$(ME_HIP_LIB=$lib timeout -k 10 160 python3 bench.py --config 8k --steps 3 --warmup 1 $C | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['kernel_ms'],3), d['parity'])")
    echo "rep $rep $lib 4k16 $r4 8k16 $r8" >> $OUT
  done
done
bash tools/dbg/r04s.sh
# SQ issue counters of the batched 1080p flow kernel and the 8K item kernel
for g in "SQ_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  COUNTERS="$g" VARIANTS="none" bash tools/dbg/pmc_variants.sh r04t_sq_1080p --steps 10 --warmup 2 --no-cpu --no-stream --no-4k --no-single --no-ssd >> gpurun_out/r04t_sq.txt 2>&1
  COUNTERS="$g" VARIANTS="none" bash tools/dbg/pmc_variants.sh r04t_sq_8k --config 8k --steps 1 --warmup 0 --no-cpu --no-stream --no-4k --no-single --no-ssd >> gpurun_out/r04t_sq.txt 2>&1
done
