set -e
mkdir -p gpurun_out
for f in 8 16; do
  timeout -k 10 300 python -u tools/stripe_sweep.py --config 1080p --frames $f --ranks 1,2,4,8 --iters 20 >> gpurun_out/r03ag_stripe_sweep_1080p.jsonl
done
cat gpurun_out/r03ag_stripe_sweep_1080p.jsonl
