set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05v}
export TMPDIR=/tmp
for F in 1 16; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_kt_f$F -o run --output-format csv -- python3 tools/ssd_ab.py --frames $F --configs 1080p,4k --tag f$F --ms 200 > gpurun_out/${T}_kt_f$F.log 2>&1; rc=$?; echo "kt $F rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
  find gpurun_out/${T}_kt_f$F -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-220
done
