set -e
mkdir -p gpurun_out
export ME_HIP_LIB=libme_hip_tune.so
run() { timeout -k 10 120 python -u tools/dbg/flow_fair_ab.py >> gpurun_out/r03ab_fair_sweep.jsonl 2>> gpurun_out/r03ab.err; }
ME_FAIR=0 ME_FLOW_ONE=0 run
for t in 8,16 16,32 24,40 32,48 40,56 48,56; do ME_FAIR=1 ME_FAIR_T=$t ME_FLOW_ONE=1 run; done
ME_FAIR=1 ME_FAIR_T=40,56 ME_FLOW_ONE=0 run
for t in 16,32 24,40 40,56; do AB_FRAMES=16 ME_FAIR=1 ME_FAIR_T=$t ME_FLOW_ONE=1 run; done
AB_FRAMES=16 ME_FAIR=0 ME_FLOW_ONE=0 run
cat gpurun_out/r03ab_fair_sweep.jsonl
