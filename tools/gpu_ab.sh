#!/bin/bash
# A/B kernel timing + PMC counters on one GPU box.  Usage: tools/gpu_ab.sh "<variant libs...>" [pmc]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for lib in $1; do
  tag=$(basename "$lib" .so)
  VAMP_AMD_LIB=$PWD/$lib timeout -k 10 300 python tools/kbench.py --edges 1048576 --reps 5 --tag "$tag" > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "kbench $tag failed"; tail -20 gpurun_out/ab/$tag.err; exit 1; }
  cat gpurun_out/ab/$tag.json
done
if [ "$2" = "pmc" ]; then
  lib=$(echo $1 | awk '{print $1}')
  rocprofv3 -L > gpurun_out/ab/counters.txt 2>&1 || true
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_WAIT_ANY SQ_INST_CYCLES_SALU" ${PMC_EXTRA:-}; do
    i=$((i+1))
    VAMP_AMD_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "panda_validate|panda_fkcc" -d gpurun_out/ab/pmc$i -o pmc --output-format csv -- python3 tools/kbench.py --edges 262144 --reps 1 --tag pmc > gpurun_out/ab/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 gpurun_out/ab/pmc$i.log; exit 1; }
  done
fi
echo done
