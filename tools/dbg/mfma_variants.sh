# Build A/B variants of the library with me_mfma.hip switches (ME_SSD8_*):
# lib/libme_hip_<name>.so, run here on the CPU box.
# usage: bash tools/dbg/mfma_variants.sh name:-DFLAG=0,-DFLAG2=0 ...
set -e
cd "$(dirname "$0")/../../motionestimation_amd/csrc"
make -s all
for spec in "$@"; do
  name=${spec%%:*}; flags=$(echo "${spec#*:}" | tr ',' ' ')
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -I../../include $flags -c -o ../lib/obj/me_mfma_$name.o me_mfma.hip
  objs=$(for o in me_kernels me_post me_api me_plan me_stream me_io me_ssim me_mfma me_band; do [ $o = me_mfma ] || echo ../lib/obj/$o.o; done)  # the product objects only
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../lib/libme_hip_$name.so $objs ../lib/obj/me_mfma_$name.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo built libme_hip_$name.so
done
