set -e
mkdir -p gpurun_out
export ME_HIP_LIB=libme_hip_tune.so
for fair in 0 1; do for one in 0 1; do
ME_FAIR=$fair ME_FLOW_ONE=$one timeout -k 10 120 python -u tools/dbg/flow_fair_ab.py >> gpurun_out/r03aa_fair_ab.jsonl 2>> gpurun_out/r03aa.err
done; done
cat gpurun_out/r03aa_fair_ab.jsonl
