# first item staged through registers (libme_hip_reg.so, -DME_REG_FIRST) vs LDS DMA, same box
set -e
for args in "--cost sad --heights 1080 --rows 26:34 --iters 80" "--cost sad --heights 1080 --rows 17:26 --iters 80" "--cost sad --heights 1080 --rows 17:34 --iters 80" "--cost sad --width 3840 --heights 2160 --span 64 --iters 20" "--cost sad --blk 8 --span 128 --width 7680 --heights 4320 --iters 4"; do
  for rep in 1 2; do
    for lib in libme_hip.so libme_hip_reg.so; do
      r=$(ME_HIP_LIB=$lib timeout -k 10 120 python3 tools/size_sweep.py $args 2>/dev/null | grep "^{" | tail -1)
      echo "$lib $rep $args :: $r" | cut -c1-200
    done
  done
done
