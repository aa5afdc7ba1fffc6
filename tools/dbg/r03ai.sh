set -e
mkdir -p gpurun_out
O=gpurun_out/r03ai_stripe_frames.jsonl
for f in 8 16 32; do
  timeout -k 10 300 python -u tools/stripe_sweep.py --config 1080p --frames $f --ranks 1,8 --iters 20 >> $O
done
timeout -k 10 300 python -u tools/stripe_sweep.py --config 4k --frames 8 --ranks 1,8 --iters 5 >> $O
timeout -k 10 300 python -u tools/stripe_sweep.py --config 4k --frames 32 --ranks 1,8 --iters 3 >> $O
cat $O
