#!/bin/bash
# round-5 pass j: the -m gpu suite on the release build (CAPT grid build with per-leaf pruning) and on lb (the
# staged bound stage's test bits accumulated per lane, one group OR at the end), then A/B rel vs lb:
# Panda cage / set A / table_pick, CAPT (+ its environment upload = grid build), composite, Fetch edge stage
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/mr-vamp_amd/vamp_amd
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05j_gputest.log 2>&1 || { tail -30 gpurun_out/r05j_gputest.log; exit 1; }
tail -n 1 gpurun_out/r05j_gputest.log
VAMP_AMD_LIB=$L/libvampgpu_lb.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05j_gputest_lb.log 2>&1 || { tail -30 gpurun_out/r05j_gputest_lb.log; exit 1; }
echo "lb: $(tail -n 1 gpurun_out/r05j_gputest_lb.log)"
: > gpurun_out/r05j_panda.log
for r in 1 2; do
  for v in rel lb; do
    lib=$L/libvampgpu.so; [ $v != rel ] && lib=$L/libvampgpu_$v.so
    for w in "validate" "validate --edge-set A" "validate --scene table_pick" "capt" "pair"; do
      VAMP_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu > gpurun_out/r05j_line.json 2>/dev/null || { echo "$w $v failed"; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/r05j_line.json')); u=d.get('environment_upload_ms', {}).get('ms'); print(json.dumps({'tag': '$v', 'kernel': '$w', 'ms': d['ms_per_step'], 'upload_ms': u}))" | tee -a gpurun_out/r05j_panda.log
    done
  done
done
FULL=1 bash tools/ab_fetch.sh r05j rel lb
# the grid build kernels' own durations (kernel trace), both builds
for v in rel lb; do
  lib=$L/libvampgpu.so; [ $v != rel ] && lib=$L/libvampgpu_$v.so
  VAMP_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05j_capt_$v -o capt --output-format csv -- python3 bench.py --workload capt --steps 3 --warmup 1 --no-cpu > gpurun_out/r05j_capt_prof_$v.log 2>&1 || { echo "capt prof $v failed"; tail -5 gpurun_out/r05j_capt_prof_$v.log; exit 1; }
  find gpurun_out/r05j_capt_$v -name "*kernel_stats.csv" -exec grep -h "capt_grid_kernel\|capt_leaf_kernel" {} \; | cut -c1-200
done
