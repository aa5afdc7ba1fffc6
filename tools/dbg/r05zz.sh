set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zz}; export TMPDIR=/tmp
# residency of the item kernel: what the planner's launch gets, then capped
python3 - <<'PY' > gpurun_out/${T}_res.txt 2>&1
import os, sys
sys.path.insert(0, os.getcwd())
PY
for CFG in 8k 4k; do
for R in 0 4 3 2 0; do
  if [ $R = 0 ]; then E=""; else E="ME_FAST_RES=$R"; fi
  env ME_HIP_LIB=libme_hip_tune.so $E timeout -k 10 200 python3 bench.py --no-cpu --no-stream --no-4k --no-single --no-ssim --no-ssd --config $CFG --steps 3 --warmup 1 > gpurun_out/${T}_${CFG}_$R.json 2>> gpurun_out/${T}.err; rc=$?; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_${CFG}_$R.json')); print('$CFG res<=$R', round(d['ms_per_step'],3), round(d['roofline']['valu']['frac'],4), d['parity'])" | tee -a gpurun_out/${T}_ab.txt
done; done
