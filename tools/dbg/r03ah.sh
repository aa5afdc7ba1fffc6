set -e
mkdir -p gpurun_out
export ME_HIP_LIB=libme_hip_tune.so
O=gpurun_out/r03ah_same_box.jsonl
timeout -k 10 120 python -u tools/dbg/flow_fair_ab.py >> $O
ME_FAIR=0 ME_FLOW_ONE=0 timeout -k 10 120 python -u tools/dbg/flow_fair_ab.py >> $O
for f in 8 16; do
  timeout -k 10 300 python -u tools/stripe_sweep.py --config 1080p --frames $f --ranks 1,8 --iters 20 >> $O
  ME_FAIR=0 ME_FLOW_ONE=0 timeout -k 10 300 python -u tools/stripe_sweep.py --config 1080p --frames $f --ranks 1,8 --iters 20 >> $O
done
timeout -k 10 120 python -u tools/dbg/flow_fair_ab.py >> $O
rocm-smi --showclocks > gpurun_out/r03ah_clocks.txt 2>&1 || true
cat $O
