set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zc}
export TMPDIR=/tmp
bash tools/dbg/rank_pg_ab.sh $T; rc=$?; echo "rank_pg_ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_ssim_kt -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-stream --no-4k --no-single --no-ssd > gpurun_out/${T}_ssim_bench.json 2> gpurun_out/${T}_ssim_bench.err; rc=$?; echo "ssim kt rc=$rc"
find gpurun_out/${T}_ssim_kt -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200
python3 -c "import json,sys; d=json.load(open('gpurun_out/${T}_ssim_bench.json')); print(json.dumps(d.get('ssim'))[:1500])"
