# small-search plan: fold (16 groups, narrower rows) vs no fold (17 groups), same box
for rep in 1 2; do
  for f in 0 1; do
    r=$(ME_HIP_LIB=libme_hip_tune.so ME_PLAN="5,1,7,64,$f" timeout -k 10 60 python3 tools/size_sweep.py --cost sad --blk 16 --span 16 --width 352 --heights 288 --iters 100 2>/dev/null | grep "^{")
    echo "cif fold=$f $r" | cut -c1-110
    r=$(ME_HIP_LIB=libme_hip_tune.so ME_PLAN="5,1,13,256,$f" timeout -k 10 60 python3 tools/size_sweep.py --cost sad --heights 1080 --rows 17:26 --iters 100 2>/dev/null | grep "^{")
    echo "9row fold=$f $r" | cut -c1-110
    r=$(ME_HIP_LIB=libme_hip_tune.so ME_PLAN="5,1,13,256,$f" timeout -k 10 60 python3 tools/size_sweep.py --cost sad --heights 1080 --rows 26:34 --iters 100 2>/dev/null | grep "^{")
    echo "8row fold=$f $r" | cut -c1-110
  done
done
