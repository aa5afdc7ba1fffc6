set -e
mkdir -p gpurun_out
export ME_HIP_LIB=libme_hip_tune.so
for P in 1 0 1 0; do
  for C in 1080p 4k; do
    ME_PRIO=$P timeout -k 10 100 python -u tools/stripe_sweep.py --config $C --ranks 1,2,8 | sed "s/^/{\"prio\": $P, \"r\": /; s/$/}/" >> gpurun_out/r03d_prio_ab.jsonl
  done
done
ME_PRIO=1 timeout -k 10 100 python -u tools/stripe_sweep.py --config 8k --ranks 1,8 | sed "s/^/{\"prio\": 1, \"r\": /; s/$/}/" >> gpurun_out/r03d_prio_ab.jsonl
ME_PRIO=0 timeout -k 10 100 python -u tools/stripe_sweep.py --config 8k --ranks 1,8 | sed "s/^/{\"prio\": 0, \"r\": /; s/$/}/" >> gpurun_out/r03d_prio_ab.jsonl
unset ME_HIP_LIB
timeout -k 10 100 python -u tools/wave_stamps.py 1080p 17:26 > gpurun_out/r03d_wave_stamps_prio.txt 2>&1
