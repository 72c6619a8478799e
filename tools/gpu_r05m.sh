#!/bin/bash
# round-5 pass m: the composite's arm passes with the Panda's mid-sphere tests in their validate tails (pm) vs rel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/mr-vamp_amd/vamp_amd
VAMP_AMD_LIB=$L/libvampgpu_pm.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pair.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05m_pair_pm.log 2>&1 || { tail -20 gpurun_out/r05m_pair_pm.log; exit 1; }
echo "pm parity: $(tail -n 1 gpurun_out/r05m_pair_pm.log)"
: > gpurun_out/r05m_pair.log
for r in 1 2 3; do
  for v in rel pm; do
    lib=$L/libvampgpu.so; [ $v != rel ] && lib=$L/libvampgpu_$v.so
    VAMP_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload pair --steps 20 --warmup 3 --no-cpu > gpurun_out/r05m_line.json 2>/dev/null || { echo "pair $v failed"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r05m_line.json')); print(json.dumps({'tag': '$v', 'kernel': 'pair', 'ms': d['ms_per_step']}))" | tee -a gpurun_out/r05m_pair.log
  done
done
