# A/B two in-tree library builds on one box: rocprof kernel averages AND the
# FETCH_SIZE / WRITE_SIZE PMC passes (own passes) per build.
#   AB_LIBS="libme_hip_base.so libme_hip.so" SWEEP_ARGS="..." bash tools/dbg/ab_fetch.sh
R=$GRAFT_REPO_ROOT
for lib in ${AB_LIBS:-libme_hip_base.so libme_hip.so}; do
  d=gpurun_out/abf_${lib}
  for pass in kt FETCH_SIZE WRITE_SIZE; do
    if [ $pass = kt ]; then opt="--kernel-trace --stats"; else opt="--pmc $pass"; fi
    (cd /tmp && ME_HIP_LIB=$lib timeout -k 10 120 rocprofv3 $opt -d $R/$d/$pass -o run --output-format csv -- python3 $R/tools/size_sweep.py ${SWEEP_ARGS} > /dev/null 2>&1) || exit 1
  done
  python3 - "$d" "$lib" <<'PY'
import csv, glob, sys, collections
d, lib = sys.argv[1], sys.argv[2]
for f in glob.glob(d + "/kt/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(lib, "time_us", r["Name"][:48], round(float(r["AverageNs"]) / 1e3, 2))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = collections.defaultdict(list)
    for f in glob.glob(d + f"/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == c:
                acc[r["Kernel_Name"][:48]].append(float(r["Counter_Value"]))
    for k, v in acc.items():  # KiB per dispatch (FETCH_SIZE: x2 on gfx950, MI355X_MICROARCH.md)
        mb = sum(v) / len(v) * 1024 / 1e6 * (2 if c == "FETCH_SIZE" else 1)
        print(lib, c, "MB_per_dispatch", k, round(mb, 2), "n", len(v))
PY
done
