set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 120 python3 tools/bw_stamps.py 1080p 16 > gpurun_out/r05c_bw_stamps.txt 2>&1; rc=$?; cat gpurun_out/r05c_bw_stamps.txt; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python3 tools/bw_stamps.py 1080p 1 >> gpurun_out/r05c_bw_stamps.txt 2>&1; rc=$?; case $rc in 0|1) ;; *) exit $rc;; esac
for P in auto prepass lean; do
  ME_PATH=$P timeout -k 10 200 python3 tools/ssd_ab.py --frames 1,16 --configs 1080p,4k --tag $P >> gpurun_out/r05c_ssd_ab.jsonl 2>> gpurun_out/r05c_ssd_ab.err; rc=$?; echo "$P rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done
cat gpurun_out/r05c_ssd_ab.jsonl
