# Round 6: band-walk with re-centred terms (w' = r - 128: no v_not in the S2 steps, keys by v_mad_i32_i24), unconditional P0 stores, uneven segments -- parity, timing, stamps.
# Round 6: band-walk producers claim slots without blocking, partial-row search on the searcher waves -- parity, timing, stamps.
# batched timing (A/B against the prepass pair), producer stamps.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_ctx_path.py tests/test_gpu_bench_batch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06f_pytest.log 2>&1
O=gpurun_out/r06f_ssd_ab.jsonl
: > $O
ME_PATH=lean timeout -k 10 120 python3 tools/ssd_ab.py --frames 1,16 --ms 300 --tag lean >> $O 2>>gpurun_out/r06f_err.log
ME_PATH=prepass timeout -k 10 120 python3 tools/ssd_ab.py --frames 1,16 --ms 300 --tag prepass >> $O 2>>gpurun_out/r06f_err.log
ME_PATH=lean timeout -k 10 120 python3 tools/bw_stamps.py 1080p 1 > gpurun_out/r06f_stamps_1080p_f1.txt 2>&1
ME_PATH=lean timeout -k 10 120 python3 tools/bw_stamps.py 1080p 16 > gpurun_out/r06f_stamps_1080p_f16.txt 2>&1
