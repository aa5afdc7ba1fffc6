set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zz2}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/${T}_pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1; echo smoke rc=$?
timeout -k 10 400 python bench.py > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.err; echo bench rc=$?
python3 -c "import json; d=json.load(open('gpurun_out/bench_${T}.json')); print(d['value'], d['ms_per_step'], d['roofline']['valu']['frac'], d['single_frame']['kernel_ms'], d['ssd_mfma']['kernel_ms'], d['ssd_mfma']['roofline']['frac'], d['host_stream']['pinned']['pairs_per_s'], d['host_stream']['pageable']['pairs_per_s'], d['parity'])"
