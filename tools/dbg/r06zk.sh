# Round 6: band-walk segment plans with a longer first / last segment (1080p
# one frame: 10 + 6 x 8 + 9 rows, 12 bands worst, against 8 x 9 uniform, 13) --
# band-walk / SSD parity tests on this build, then A/B on one box: the tuning
# build uniform (ME_BW_SEGFIRST=0) against this build, 1080p and 4K one frame.
# (Second run, r06zl: the uniform plan as a product-build variant,
# -DME_BW_SEG_UNIFORM, against this build: the tuning build itself is slower.)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_ctx_path.py tests/test_gpu_fullframe.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06zk_pytest.log 2>&1
O=gpurun_out/r06zk_bw_seg.jsonl
: > $O
for rep in 1 2 3; do
  ME_BW_SEGFIRST=0 ME_HIP_LIB=libme_hip_tune.so timeout -k 10 240 python3 tools/ssd_ab.py --frames 1 --tag uniform >> $O 2>>gpurun_out/r06zk_err.log
  timeout -k 10 240 python3 tools/ssd_ab.py --frames 1 --tag firstlast >> $O 2>>gpurun_out/r06zk_err.log
done
