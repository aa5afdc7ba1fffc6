# SQ counter passes over one kernel of the search (GPU box, repo root):
#   [SQ_ARGS="size_sweep.py shape args"] bash tools/sq_counters.sh [cost] [kernel-name filter]   (default: sad me_fast, 1080p)
# One rocprofv3 --pmc pass per group (slot limits: MI355X_MICROARCH.md), each
# under its own time limit; summary -> gpurun_out/sq/summary.txt
set -e
COST=${1:-sad}
FILT=${2:-me_fast}
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/sq
i=0
for g in "SQ_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
         "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
         "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU" \
         "SQ_INSTS_VALU_MFMA_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $g -T -d $R/gpurun_out/sq/p$i -o out --output-format csv -- python3 $R/tools/size_sweep.py --cost $COST ${SQ_ARGS:---heights 1080} --iters ${ITERS:-10} > $R/gpurun_out/sq/log$i.txt 2>&1 || echo "pass $i failed: $g"
done
python3 $R/tools/pmc_counters.py $R/gpurun_out/sq $FILT > $R/gpurun_out/sq/summary.txt
cat $R/gpurun_out/sq/summary.txt
