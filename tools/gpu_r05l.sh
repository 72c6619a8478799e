#!/bin/bash
# round-5 pass l: A/B of the kNN visiting order (ko: nearest-first tiles and super-tiles) on the Fetch edge stage,
# and of the composite's combined inter-arm bound kernel at 6 / 7 waves/EU (pb6, pb7)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/mr-vamp_amd/vamp_amd
for v in ko1 ko; do VAMP_AMD_LIB=$L/libvampgpu_$v.so timeout -k 10 200 python tools/knn_debug.py 200000 > gpurun_out/r05l_knn_debug_$v.log 2>&1 || { tail -5 gpurun_out/r05l_knn_debug_$v.log; exit 1; }; grep -v amdgpu.ids gpurun_out/r05l_knn_debug_$v.log | head -2; done
for v in pb6 pb7; do
  VAMP_AMD_LIB=$L/libvampgpu_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pair.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05l_pair_$v.log 2>&1 || { tail -20 gpurun_out/r05l_pair_$v.log; exit 1; }
  echo "$v pair parity: $(tail -n 1 gpurun_out/r05l_pair_$v.log)"
done
: > gpurun_out/r05l_pair.log
for r in 1 2; do
  for v in rel pb6 pb7; do
    lib=$L/libvampgpu.so; [ $v != rel ] && lib=$L/libvampgpu_$v.so
    VAMP_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload pair --steps 20 --warmup 3 --no-cpu > gpurun_out/r05l_line.json 2>/dev/null || { echo "pair $v failed"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r05l_line.json')); print(json.dumps({'tag': '$v', 'kernel': 'pair', 'ms': d['ms_per_step']}))" | tee -a gpurun_out/r05l_pair.log
  done
done
FULL=1 bash tools/ab_fetch.sh r05l rel ko1 ko
