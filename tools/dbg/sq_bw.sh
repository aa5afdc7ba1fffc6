# SQ counter passes over the band-walk (ME_PATH=auto) and block-major
# (ME_PATH=prepass) SSD kernels: 16-frame 1080p batches of tools/ssd_ab.py.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for P in auto prepass; do
  mkdir -p $R/gpurun_out/sq_$P
  i=0
  for g in "SQ_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
           "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU" \
           "SQ_INSTS_VALU_MFMA_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC"; do
    i=$((i+1))
    ME_PATH=$P timeout -s KILL 90 rocprofv3 --pmc $g -T -d $R/gpurun_out/sq_$P/p$i -o out --output-format csv -- python3 $R/tools/ssd_ab.py --frames 16 --configs 1080p --ms 100 > $R/gpurun_out/sq_$P/log$i.txt 2>&1 || echo "pass $i failed: $g"
  done
done
python3 $R/tools/pmc_counters.py $R/gpurun_out/sq_auto me_mfma_bw > $R/gpurun_out/sq_auto/summary.txt
python3 $R/tools/pmc_counters.py $R/gpurun_out/sq_prepass me_mfma_bm16 > $R/gpurun_out/sq_prepass/summary.txt
cat $R/gpurun_out/sq_auto/summary.txt $R/gpurun_out/sq_prepass/summary.txt
