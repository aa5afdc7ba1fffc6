# Round 6: band-walk A/B on one box -- round-5 library against this round's
# changes one at a time (tools/dbg/bw_variants.sh builds), lean path, 1080p
# and 4K, 1 and 16 frames per call; two interleaved repetitions.
set -e
mkdir -p gpurun_out
O=gpurun_out/r06g_bw_ab.jsonl
: > $O
for rep in 1 2; do
  for lib in r5 old3 nb0 pipe0 even cur; do
    L=libme_hip_$lib.so; [ $lib = cur ] && L=libme_hip.so
    ME_HIP_LIB=$L ME_PATH=lean timeout -k 10 120 python3 tools/ssd_ab.py --frames 1,16 --ms 200 --tag "$lib" >> $O 2>>gpurun_out/r06g_err.log
  done
done
