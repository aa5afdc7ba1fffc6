# SSD 16x16 at 1080p: block-major vs 4x4-block-tile MFMA kernel over the range S
for S in 2 4 8 12 16 24 32 48 64; do for bm in 1 0; do
  r=$(ME_HIP_LIB=libme_hip_tune.so ME_MFMA_BM=$bm timeout -k 10 60 python tools/size_sweep.py --cost ssd --span $S --heights 1080 --iters 30 | tail -1) || exit 1
  echo "S=$S bm=$bm $r"
done; done
