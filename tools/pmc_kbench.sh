#!/bin/bash
# PMC passes over tools/kbench.py for kernels matching a regex.  Usage: tools/pmc_kbench.sh <regex> [edges]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
RX=$1
E=${2:-262144}
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQC_ICACHE_MISSES SQC_ICACHE_HITS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "$RX" -d gpurun_out/pmc/pmc$i -o pmc --output-format csv -- python3 tools/kbench.py --edges $E --reps 1 --tag pmc > gpurun_out/pmc/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 gpurun_out/pmc/pmc$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc
