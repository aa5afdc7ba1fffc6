set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zi}; export TMPDIR=/tmp
C="--no-cpu --no-stream --no-4k --no-single --no-ssim --cost ssd --config 8k --steps 4 --warmup 1"
for V in libme_hip.so libme_hip_v_old.so libme_hip_v_s16.so libme_hip_v_s64.so; do
  ME_HIP_LIB=$V timeout -k 10 200 python3 bench.py $C > gpurun_out/${T}_$V.json 2> gpurun_out/${T}_$V.err; rc=$?; echo "$V bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${T}_$V.json')); print('$V', d['ms_per_step'], d.get('kernel_ms'), d['parity'] if 'parity' in d else '')"
  ME_HIP_LIB=$V timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}_pmc_$V -o run --output-format csv -- python3 bench.py $C > gpurun_out/${T}_pmc_$V.log 2>&1; rc=$?; echo "$V pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/dbg/pmc_kernel_sum.py gpurun_out/${T}_pmc_$V FETCH_SIZE
done
