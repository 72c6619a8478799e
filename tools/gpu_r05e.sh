#!/bin/bash
# round-5 pass e: the -m gpu suite on the release build (block-cooperative kNN default), kNN check at 200k,
# kNN kernel / Fetch children occupancy A/B incl. the full-size edge stage, CAPT EXT children occupancy, pair
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/mr-vamp_amd/vamp_amd
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05e_gputest.log 2>&1 || { tail -30 gpurun_out/r05e_gputest.log; exit 1; }
tail -n 1 gpurun_out/r05e_gputest.log
timeout -k 10 200 python tools/knn_debug.py 200000 2>&1 | grep -v amdgpu.ids | head -3 || exit 1
: > gpurun_out/r05e_capt.log
for r in 1 2; do
  for v in rel e5; do
    lib=$L/libvampgpu.so; [ $v != rel ] && lib=$L/libvampgpu_$v.so
    VAMP_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload capt --steps 10 --warmup 2 --no-cpu > gpurun_out/r05e_line.json 2>/dev/null || { echo "capt $v failed"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r05e_line.json')); print(json.dumps({'tag': '$v', 'kernel': 'capt', 'ms': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms']}))" | tee -a gpurun_out/r05e_capt.log
  done
done
timeout -k 10 300 python bench.py --workload pair --steps 10 --warmup 2 --no-cpu > gpurun_out/r05e_pair.json 2>/dev/null || { echo "pair failed"; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05e_pair.json')); print('pair', d['ms_per_step'], d['value'])"
FULL=1 bash tools/ab_fetch.sh r05e rel rel:VAMP_AMD_KNN_COOP=0 rel:VAMP_AMD_KNN_COOP=8 fa fb
