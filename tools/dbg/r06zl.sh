# Round 6: band-walk segment plans, product builds on one box: uniform
# splits (-DME_BW_SEG_UNIFORM) against a longer first / last segment (this
# build), 1080p and 4K one frame, four rounds.
set -e
mkdir -p gpurun_out
O=gpurun_out/r06zl_bw_seg.jsonl
: > $O
for rep in 1 2 3 4; do
  ME_HIP_LIB=libme_hip_uniform.so timeout -k 10 240 python3 tools/ssd_ab.py --frames 1 --tag uniform >> $O 2>>gpurun_out/r06zl_err.log
  timeout -k 10 240 python3 tools/ssd_ab.py --frames 1 --tag firstlast >> $O 2>>gpurun_out/r06zl_err.log
done
