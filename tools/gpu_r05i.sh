#!/bin/bash
# round-5 pass i: the -m gpu suite on the release build (Fetch mid spheres for validate heads + tails, three kNN
# tiles in flight, the composite's inter-arm chunks from one bound kernel), then A/B:
#   composite: rel vs pb5 (its combined bound kernel at 5 waves/EU) vs pb0 (one bound kernel per chunk)
#   Fetch edge stage 100k + 2.68M: rel vs fm3 (mid spheres for the sampler too) vs kd4 (four kNN tiles)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/mr-vamp_amd/vamp_amd
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05i_gputest.log 2>&1 || { tail -30 gpurun_out/r05i_gputest.log; exit 1; }
tail -n 1 gpurun_out/r05i_gputest.log
for v in rel kd4; do
  lib=$L/libvampgpu.so; [ $v != rel ] && lib=$L/libvampgpu_$v.so
  VAMP_AMD_LIB=$lib timeout -k 10 200 python tools/knn_debug.py 200000 > gpurun_out/r05i_knn_debug_$v.log 2>&1 || { tail -5 gpurun_out/r05i_knn_debug_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/r05i_knn_debug_$v.log | head -2
done
for v in pb5 pb0; do
  VAMP_AMD_LIB=$L/libvampgpu_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pair.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05i_pair_$v.log 2>&1 || { tail -20 gpurun_out/r05i_pair_$v.log; exit 1; }
  echo "$v pair parity: $(tail -n 1 gpurun_out/r05i_pair_$v.log)"
done
: > gpurun_out/r05i_pair.log
for r in 1 2; do
  for v in rel pb5 pb0; do
    lib=$L/libvampgpu.so; [ $v != rel ] && lib=$L/libvampgpu_$v.so
    VAMP_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload pair --steps 20 --warmup 3 --no-cpu > gpurun_out/r05i_line.json 2>/dev/null || { echo "pair $v failed"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r05i_line.json')); print(json.dumps({'tag': '$v', 'kernel': 'pair', 'ms': d['ms_per_step'], 'parity': d.get('parity')}))" | tee -a gpurun_out/r05i_pair.log
  done
done
FULL=1 bash tools/ab_fetch.sh r05i rel fm3 kd4
