set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05r}
for A in 0 64 128 192 1 2; do
  ME_HIP_LIB=libme_hip_tune.so ME_BW_ABL=$A timeout -k 10 100 python3 tools/ssd_ab.py --frames 16 --configs 1080p --tag abl$A --ms 300 >> gpurun_out/${T}_abl.jsonl 2>> gpurun_out/${T}_abl.err; rc=$?; echo "abl $A rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done
for P in prepass auto; do
  ME_PATH=$P timeout -k 10 100 python3 tools/ssd_ab.py --frames 16 --configs 1080p,4k --tag $P --ms 300 >> gpurun_out/${T}_abl.jsonl 2>> gpurun_out/${T}_abl.err; rc=$?; echo "path $P rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done
cat gpurun_out/${T}_abl.jsonl
