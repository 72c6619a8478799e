#!/bin/bash
# Step profiles of every bench workload's step (tools/pmc_drive.py): kernel trace + stats, then one
# PMC pass per counter group (SQ <= 8 per pass; FETCH_SIZE and WRITE_SIZE in passes of their own), then
# tools/pmc_report.py -> gpurun_out/prof/<W>.json.   usage: bash tools/prof_step.sh W [W ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
for W in "$@"; do
  D=gpurun_out/prof/$W
  rm -rf $D && mkdir -p $D
  timeout -k 10 300 python3 tools/pmc_drive.py prep --workload $W > $D/prep.log 2>&1 || { echo "prep $W failed"; tail -20 $D/prep.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/trace -o trace --output-format csv -- \
      python3 tools/pmc_drive.py run --workload $W --calls 2 > $D/trace.log 2>&1 || { echo "trace $W failed"; tail -20 $D/trace.log; exit 1; }
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD" \
             "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $set -d $D/pmc_$i -o pmc --output-format csv -- \
        python3 tools/pmc_drive.py run --workload $W --calls 2 > $D/pmc_$i.log 2>&1 || { echo "pmc $W pass $i failed"; tail -5 $D/pmc_$i.log; exit 1; }
  done
  python3 tools/pmc_report.py $W $D gpurun_out/prof/$W.json || exit 1
  # keep the summaries only (gpurun copies back <= 64 MiB): the kernel stats CSV and the record
  cp $(find $D/trace -name "*kernel_stats.csv" | head -1) gpurun_out/prof/${W}_kernel_stats.csv 2>/dev/null
  rm -rf $D/trace $D/pmc_*/
done
echo prof done
