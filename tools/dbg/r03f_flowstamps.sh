set -e
mkdir -p gpurun_out
for R in 17:26 9:17 0:17; do
  echo "== rows $R" >> gpurun_out/r03f_flow_stamps.txt
  timeout -k 10 100 python -u tools/flow_stamps.py $R >> gpurun_out/r03f_flow_stamps.txt 2>&1
done
