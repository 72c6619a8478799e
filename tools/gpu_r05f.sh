#!/bin/bash
# round-5 pass f: the -m gpu suite on the release build (obstacle bounding-sphere prefilter, grazing-contact
# parity), then release vs the previous build (libvampgpu_old.so: no prefilter) on the Fetch edge stage
# (100k and 2.68M vertices) and on the Panda cage / table_pick and composite steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/mr-vamp_amd/vamp_amd
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05f_gputest.log 2>&1 || { tail -30 gpurun_out/r05f_gputest.log; exit 1; }
tail -n 1 gpurun_out/r05f_gputest.log
: > gpurun_out/r05f_panda.log
for r in 1 2; do
  for v in rel old; do
    lib=$L/libvampgpu.so; [ $v != rel ] && lib=$L/libvampgpu_$v.so
    for w in "validate" "validate --scene table_pick" "pair"; do
      VAMP_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu > gpurun_out/r05f_line.json 2>/dev/null || { echo "$w $v failed"; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/r05f_line.json')); print(json.dumps({'tag': '$v', 'kernel': '$w', 'ms': d['ms_per_step']}))" | tee -a gpurun_out/r05f_panda.log
    done
  done
done
FULL=1 bash tools/ab_fetch.sh r05f rel old
