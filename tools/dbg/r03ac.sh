set -e
mkdir -p gpurun_out
export ME_HIP_LIB=libme_hip_tune.so
run() { timeout -k 10 120 python -u tools/dbg/flow_fair_ab.py >> gpurun_out/r03ac_fair_sweep.jsonl 2>> gpurun_out/r03ac.err; }
ME_FAIR=0 ME_FLOW_ONE=0 run
for t in 1,2 4,8 8,16 8,32 12,24 1,255; do ME_FAIR=1 ME_FAIR_T=$t ME_FLOW_ONE=1 run; done
ME_FAIR=1 ME_FAIR_T=8,16 ME_FLOW_ONE=0 run
ME_FAIR=1 ME_FAIR_T=4,8 ME_FLOW_ONE=0 run
cat gpurun_out/r03ac_fair_sweep.jsonl
