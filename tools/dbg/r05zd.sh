set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zd}
run() { echo "== $*" >> gpurun_out/${T}_hs.txt; env ME_HIP_LIB=libme_hip_tune.so "$@" timeout -k 10 120 python3 tools/dbg/hs_probe.py none >> gpurun_out/${T}_hs.txt 2>&1; rc=$?; echo "$* rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac; }
run ME_STREAM_X=0
run ME_STREAM_BATCH=12
run ME_STREAM_BATCH=16
run ME_STREAM_AHEAD=3
run ME_STREAM_AHEAD=4
run ME_STREAM_COOL=4
cat gpurun_out/${T}_hs.txt
