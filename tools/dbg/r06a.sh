# Round 6: single-frame 16x16 SSD on the band-walk kernel -- segment-length
# sweep (tuning build), partial-row on/off, and per-phase stamps.
set -e
mkdir -p gpurun_out
O=gpurun_out/r06a_seg_sweep.jsonl
: > $O
for seg in 0 5 7 9 12 17 23 34 67; do
  if [ $seg = 0 ]; then E=""; else E="ME_BW_SEG=$seg"; fi
  env ME_HIP_LIB=libme_hip_tune.so ME_PATH=lean $E timeout -k 10 120 python3 tools/ssd_ab.py --frames 1 --configs 1080p --ms 200 --tag "lean_seg$seg" >> $O 2>>gpurun_out/r06a_err.log
done
env ME_HIP_LIB=libme_hip_tune.so ME_PATH=lean ME_BW_HB=0 timeout -k 10 120 python3 tools/ssd_ab.py --frames 1 --configs 1080p --ms 200 --tag lean_hb0 >> $O 2>>gpurun_out/r06a_err.log
for seg in 0 34 45 68; do
  if [ $seg = 0 ]; then E=""; else E="ME_BW_SEG=$seg"; fi
  env ME_HIP_LIB=libme_hip_tune.so ME_PATH=lean $E timeout -k 10 120 python3 tools/ssd_ab.py --frames 1 --configs 4k --ms 300 --tag "lean_seg$seg" >> $O 2>>gpurun_out/r06a_err.log
done
ME_PATH=lean timeout -k 10 120 python3 tools/bw_stamps.py 1080p 1 > gpurun_out/r06a_stamps_1080p_f1.txt 2>&1
ME_PATH=lean timeout -k 10 120 python3 tools/bw_stamps.py 1080p 16 > gpurun_out/r06a_stamps_1080p_f16.txt 2>&1
