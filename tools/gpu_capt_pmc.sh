#!/bin/bash
# CAPT (BASELINE configs[2]) counter passes on the GPU box: kernel-trace stats of tools/kbench_capt.py,
# then one PMC pass each for FETCH_SIZE, WRITE_SIZE and the L2 hit/miss pair (rocprofv3 does not
# split counters over passes).  Output under gpurun_out/capt_<tag>_*; tools/pmc_summary.py reads them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r02}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/capt_${T}_trace -o capt --output-format csv \
    -- python3 tools/kbench_capt.py > gpurun_out/capt_${T}_trace.log 2>&1 || exit 1
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "bound_kernel|children_kernel|capt" \
        -d gpurun_out/capt_${T}_pmc$i -o pmc --output-format csv -- python3 tools/kbench_capt.py \
        > gpurun_out/capt_${T}_pmc$i.log 2>&1 || exit $((10 + i))
done
echo done
