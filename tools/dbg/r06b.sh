# Round 6: single-frame band-walk -- producer issue priority (tuning build
# ME_BW_ABL=16 whole walk / 32 first ring) x segment length; stamps with the
# per-workgroup lifetimes.
set -e
mkdir -p gpurun_out
O=gpurun_out/r06b_prio_sweep.jsonl
: > $O
for abl in 0 16 32; do
  for seg in 0 5 7 12; do
    E="ME_BW_ABL=$abl"; [ $seg != 0 ] && E="$E ME_BW_SEG=$seg"
    env ME_HIP_LIB=libme_hip_tune.so ME_PATH=lean $E timeout -k 10 120 python3 tools/ssd_ab.py --frames 1 --configs 1080p --ms 200 --tag "abl${abl}_seg$seg" >> $O 2>>gpurun_out/r06b_err.log
  done
  env ME_HIP_LIB=libme_hip_tune.so ME_PATH=lean ME_BW_ABL=$abl timeout -k 10 120 python3 tools/ssd_ab.py --frames 1,16 --configs 4k --ms 300 --tag "abl${abl}" >> $O 2>>gpurun_out/r06b_err.log
  env ME_HIP_LIB=libme_hip_tune.so ME_PATH=lean ME_BW_ABL=$abl timeout -k 10 120 python3 tools/ssd_ab.py --frames 16 --configs 1080p --ms 300 --tag "abl${abl}" >> $O 2>>gpurun_out/r06b_err.log
done
ME_PATH=lean timeout -k 10 120 python3 tools/bw_stamps.py 1080p 1 > gpurun_out/r06b_stamps_1080p_f1.txt 2>&1
ME_PATH=lean timeout -k 10 120 python3 tools/bw_stamps.py 4k 1 > gpurun_out/r06b_stamps_4k_f1.txt 2>&1
