set -e
mkdir -p gpurun_out
O=gpurun_out/r03aj_flow_stamps.txt
for b in batch8 batch32 batch16; do
echo "== $b" >> $O
FLOW_STAMPS_SAVE=gpurun_out/r03aj_flow_$b.npy timeout -k 10 100 python -u tools/flow_stamps.py $b 2>&1 | grep -v amdgpu.ids >> $O
done
cat $O
