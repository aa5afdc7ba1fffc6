# A/B two in-tree library builds on one box: rocprof kernel averages per build
for lib in ${AB_LIBS:-libme_hip_old.so libme_hip_new.so}; do
  for rep in 1 2; do
    d=gpurun_out/ab_${lib}_$rep
    (cd /tmp && ME_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$d -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/size_sweep.py ${SWEEP_ARGS:---cost ssd --heights 1080 --iters 40} > /dev/null 2>&1) || exit 1
    python3 - "$d" "$lib" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fill" not in r["Name"]:
            print(sys.argv[2], r["Name"][30:62], round(float(r["AverageNs"]) / 1e3, 2))
PY
  done
done
