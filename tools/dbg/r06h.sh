# Round 6: single frames on the band-walk kernel by default -- MFMA / stream /
# per-context tests, then one-box A/B of the automatic path (band-walk) against
# the prepass pair and the round-5 library, and stamps with workgroup start /
# end times.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_ctx_path.py tests/test_gpu_bench_batch.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06h_pytest.log 2>&1
O=gpurun_out/r06h_ssd_ab.jsonl
: > $O
for rep in 1 2; do
  ME_PATH=auto timeout -k 10 120 python3 tools/ssd_ab.py --frames 1,16 --ms 250 --tag auto >> $O 2>>gpurun_out/r06h_err.log
  ME_PATH=prepass timeout -k 10 120 python3 tools/ssd_ab.py --frames 1,16 --ms 250 --tag prepass >> $O 2>>gpurun_out/r06h_err.log
  ME_HIP_LIB=libme_hip_r5.so ME_PATH=auto timeout -k 10 120 python3 tools/ssd_ab.py --frames 1,16 --ms 250 --tag r5auto >> $O 2>>gpurun_out/r06h_err.log
done
timeout -k 10 120 python3 tools/bw_stamps.py 1080p 1 > gpurun_out/r06h_stamps_1080p_f1.txt 2>&1
timeout -k 10 120 python3 tools/bw_stamps.py 4k 1 > gpurun_out/r06h_stamps_4k_f1.txt 2>&1
