set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zr}; export TMPDIR=/tmp
for i in 1 2; do timeout -k 10 120 python3 tools/dbg/stream_trace.py 64 > gpurun_out/${T}_times$i.txt 2>&1 || exit $?; cat gpurun_out/${T}_times$i.txt | grep pairs; done
TRACE_ONCE=1 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${T}_trace -o run -- python3 tools/dbg/stream_trace.py 64 > gpurun_out/${T}_trace.log 2>&1; echo trace rc=$?
grep -ci "drop\|timeout\|callback" gpurun_out/${T}_trace.log || true
