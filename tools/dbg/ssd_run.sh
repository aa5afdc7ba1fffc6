set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mfma_tests.log 2>&1 || { tail -40 gpurun_out/mfma_tests.log; exit 1; }
tail -2 gpurun_out/mfma_tests.log
for c in 1080p 4k; do timeout -k 10 120 python bench.py --cost ssd --config $c --no-cpu --no-stream --steps 20 > gpurun_out/b_ssd_$c.json 2>gpurun_out/b_ssd_$c.err || exit 1; done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for c in 1080p 4k; do timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ssd_$c -o run --output-format csv -- python3 $R/bench.py --cost ssd --config $c --no-cpu --no-stream --steps 20 > $R/gpurun_out/prof_ssd_$c.log 2>&1 || exit 1; done
python3 -c "
import json
for c in ['1080p','4k']:
    d=json.load(open('$R/gpurun_out/b_ssd_%s.json'%c)); print(c, 'kernel_ms', round(d['kernel_ms'],4), 'cand/s %.3e'%d['value'])
"
