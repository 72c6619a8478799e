#!/bin/bash
# PMC passes (one counter set per run) over the kNN kernel (prm_edges bench) and the staged
# children/bound kernels (validate bench): instruction mix, waits, occupancy.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $set --kernel-include-regex "knn_kernel" -d gpurun_out/pmc2/knn$i -o pmc --output-format csv -- python3 bench.py --workload prm_edges --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc2/knn$i.log 2>&1 || { echo "knn pass $i failed"; tail -5 gpurun_out/pmc2/knn$i.log; }
  timeout -s KILL 180 rocprofv3 --pmc $set --kernel-include-regex "children_kernel|bound_kernel" -d gpurun_out/pmc2/val$i -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu --no-fk-leg > gpurun_out/pmc2/val$i.log 2>&1 || { echo "val pass $i failed"; tail -5 gpurun_out/pmc2/val$i.log; }
done
echo done
