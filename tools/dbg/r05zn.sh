set -o pipefail; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T=${TAG:-r05zn}; export TMPDIR=/tmp
timeout -k 10 120 python3 tools/bw_stamps.py 1080p 16 > gpurun_out/${T}_stamps.txt 2>&1; echo stamps rc=$?; cat gpurun_out/${T}_stamps.txt | tail -22
for A in 0 1 2 4 64 128; do
  ME_HIP_LIB=libme_hip_tune.so ME_BW_ABL=$A timeout -k 10 100 python3 tools/ssd_ab.py --frames 16 --configs 1080p --tag abl$A --ms 300 >> gpurun_out/${T}_abl.jsonl 2>> gpurun_out/${T}_abl.err; rc=$?; echo "abl $A rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done
cat gpurun_out/${T}_abl.jsonl
cd /tmp
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/${T}_sq; i=0
for g in "SQ_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
         "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
         "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU" \
         "SQ_INSTS_VALU_MFMA_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $g -T -d $R/gpurun_out/${T}_sq/p$i -o out --output-format csv -- python3 $R/tools/ssd_ab.py --frames 16 --configs 1080p --ms 100 > $R/gpurun_out/${T}_sq/log$i.txt 2>&1 || { echo "pass $i failed: $g"; exit 1; }
done
python3 $R/tools/pmc_counters.py $R/gpurun_out/${T}_sq me_mfma_bw > $R/gpurun_out/${T}_sq/summary.txt; cat $R/gpurun_out/${T}_sq/summary.txt
