# Build A/B variants of the library with me_ssim.hip switches (ME_SSIM_*).
# usage: bash tools/dbg/ssim_variants.sh name:-DFLAG=0,... ...
set -e
cd "$(dirname "$0")/../../motionestimation_amd/csrc"
make -s all
for spec in "$@"; do
  name=${spec%%:*}; flags=$(echo "${spec#*:}" | tr ',' ' ')
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -I../../include -ffp-contract=off $flags -c -o ../lib/obj/me_ssim_$name.o me_ssim.hip
  objs=$(for o in me_kernels me_post me_api me_plan me_stream me_io me_ssim me_mfma me_band; do [ $o = me_ssim ] || echo ../lib/obj/$o.o; done)  # the product objects only
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../lib/libme_hip_$name.so $objs ../lib/obj/me_ssim_$name.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo built libme_hip_$name.so
done
