set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/profile_all.sh r03an
