# SSD 16x16 at 1080p, S 64..103: block-major (LP 544 above 64) vs 4x4-block tiles
for S in 64 72 80 96 103; do for bm in 1 0; do
  r=$(ME_HIP_LIB=libme_hip_tune.so ME_MFMA_BM=$bm timeout -k 10 60 python tools/size_sweep.py --cost ssd --span $S --heights 1080 --iters 20 | tail -1) || exit 1
  echo "S=$S bm=$bm $r"
done; done
