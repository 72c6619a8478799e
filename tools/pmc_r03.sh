#!/bin/bash
# Round-3 PMC passes of the headline validate call (tools/kbench.py, 2^18 cage edges, one call after
# one warm-up), one counter group per rocprofv3 run (SQ <= 8, TCC: FETCH_SIZE and WRITE_SIZE apart).
# usage: bash tools/pmc_r03.sh TAG [lib]   -> gpurun_out/pmc_TAG_<i>/ ; tools/pmc_summary.py reads them
TAG=${1:-r03}
LIB=${2:-mr-vamp_amd/vamp_amd/libvampgpu.so}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
KRE="bound_kernel|children_kernel|count_kernel|queue_kernel|plan_kernel|tail_counts|scatter_items|total64"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_WAIT_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  VAMP_AMD_LIB=$PWD/$LIB timeout -s KILL 150 rocprofv3 --pmc $set --kernel-include-regex "$KRE" \
      -d gpurun_out/pmc_${TAG}_$i -o pmc --output-format csv -- python3 tools/kbench.py --edges 262144 --reps 1 --tag pmc --only-setb \
      > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pmc pass $i ($set) failed"; tail -5 gpurun_out/pmc_${TAG}_$i.log; }
done
echo pmc done
