set -e
mkdir -p gpurun_out
O=gpurun_out/r03ak_same_box.jsonl
AB_FRAMES=16 timeout -k 10 120 python -u tools/dbg/flow_fair_ab.py >> $O
timeout -k 10 300 python -u tools/stripe_sweep.py --config 1080p --frames 16 --ranks 1 --iters 20 >> $O
AB_FRAMES=16 timeout -k 10 120 python -u tools/dbg/flow_fair_ab.py >> $O
timeout -k 10 300 python -u tools/stripe_sweep.py --config 1080p --frames 16 --ranks 1 --iters 20 >> $O
cat $O
