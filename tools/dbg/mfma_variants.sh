# Build A/B variants of the library with me_mfma.hip switches (ME_SSD8_*):
# lib/libme_hip_<name>.so, run here on the CPU box.
# usage: bash tools/dbg/mfma_variants.sh name:-DFLAG=0,-DFLAG2=0 ...
set -e
cd "$(dirname "$0")/../../motionestimation_amd/csrc"
make -s all
for spec in "$@"; do
  name=${spec%%:*}; flags=$(echo "${spec#*:}" | tr ',' ' ')
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -I../../include $flags -c -o ../lib/obj/me_mfma_$name.o me_mfma.hip
  objs=$(ls ../lib/obj/me_*.o | grep -v -E "me_mfma|_tune|_stamps")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../lib/libme_hip_$name.so $objs ../lib/obj/me_mfma_$name.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo built libme_hip_$name.so
done
