set -e
mkdir -p gpurun_out
export ME_HIP_LIB=libme_hip_tune.so
run() { timeout -k 10 120 python -u tools/dbg/flow_fair_ab.py >> gpurun_out/r03af_fair_modes.jsonl 2>> gpurun_out/r03af.err; }
for rep in 1 2; do
for f in 0 1 2 3; do ME_FAIR=$f run; done
ME_FAIR=0 ME_FLOW_ONE=0 run
done
cat gpurun_out/r03af_fair_modes.jsonl
