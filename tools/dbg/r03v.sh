set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
SWEEP_ARGS="--cost sad --heights 1080 --iters 300" AB_LIBS="libme_hip_old.so libme_hip_new.so libme_hip_old.so libme_hip_new.so" bash tools/dbg/ab.sh > gpurun_out/r03v_ab_1080p.txt 2>&1
SWEEP_ARGS="--cost sad --width 3840 --span 64 --heights 2160 --iters 30" AB_LIBS="libme_hip_old.so libme_hip_new.so" bash tools/dbg/ab.sh > gpurun_out/r03v_ab_4k.txt 2>&1
timeout -k 10 300 python -u tools/step_overhead.py --steps 4000 > gpurun_out/r03v_step_overhead.jsonl
