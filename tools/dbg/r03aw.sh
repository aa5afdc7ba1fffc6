# 8K 8x8 SAD (K = 26): strip width vs fetched bytes and time (tuning build)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for S in 16 8 4 32 0; do
  ME_HIP_LIB=libme_hip_tune.so ME_STRIP=$S timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r03aw_fetch_s$S -o run --output-format csv -- python3 tools/dbg/traffic_probe.py 8k sad 2 > /dev/null 2>&1
  ME_HIP_LIB=libme_hip_tune.so ME_STRIP=$S timeout -k 10 200 python -u tools/stripe_sweep.py --config 8k --ranks 1 --iters 4 >> gpurun_out/r03aw_time_s$S.jsonl
done
ME_HIP_LIB=libme_hip_tune.so ME_PLAN=13,8,0,256,1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r03aw_fetch_k13 -o run --output-format csv -- python3 tools/dbg/traffic_probe.py 8k sad 2 > /dev/null 2>&1
python3 - <<'PY'
import csv, glob
for d in sorted(glob.glob("gpurun_out/r03aw_fetch_*")):
    v = [float(r["Counter_Value"]) for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True)
         for r in csv.DictReader(open(f)) if r.get("Counter_Name") == "FETCH_SIZE" and "fast" in r["Kernel_Name"]]
    print(d, "MB per launch (x2)", [round(x * 1024 * 2 / 1e6, 1) for x in v])
PY
cat gpurun_out/r03aw_time_s*.jsonl
