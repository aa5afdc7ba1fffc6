set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for A in 0 1 2 4 8 3 7 15; do
  ME_HIP_LIB=libme_hip_tune.so ME_BW_ABL=$A timeout -k 10 100 python3 tools/ssd_ab.py --frames 16 --configs 1080p --tag abl$A --ms 200 >> gpurun_out/r05i_abl.jsonl 2>> gpurun_out/r05i_abl.err; rc=$?; echo "abl $A rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done
cat gpurun_out/r05i_abl.jsonl
