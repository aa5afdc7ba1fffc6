set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/sq
i=0
for g in "SQ_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $g -T -d $R/gpurun_out/sq/p$i -o out --output-format csv -- python3 $R/tools/size_sweep.py --heights 1080 --iters 10 > $R/gpurun_out/sq/log$i.txt 2>&1
done
python3 $R/tools/pmc_counters.py $R/gpurun_out/sq me_fast > $R/gpurun_out/sq/summary.txt
cat $R/gpurun_out/sq/summary.txt
