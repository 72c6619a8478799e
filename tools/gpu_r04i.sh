#!/bin/bash
# round-4 pass i: the GPU suite on the bounds-checked build, then every bench workload on the release build
# (lines kept under gpurun_out/bench_r04i_*.json) and fresh profiles of every workload's step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VAMP_AMD_LIB=$PWD/mr-vamp_amd/vamp_amd/libvampgpu_debug.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04i_gputest_debug.log 2>&1 || { tail -30 gpurun_out/r04i_gputest_debug.log; exit 1; }
tail -2 gpurun_out/r04i_gputest_debug.log
bash tools/prof_r04.sh validate validate_setA capt pair fetch_prm prm_edges || exit 1
for w in validate pair fetch_prm prm_edges capt rrtc; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 > gpurun_out/bench_r04i_$w.json 2> gpurun_out/bench_r04i_$w.err || { echo "bench $w failed"; tail -20 gpurun_out/bench_r04i_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_r04i_$w.json')); r=d.get('roofline') or {}; print('$w', d['value'], d['unit'], 'ms', d['ms_per_step'], 'kernel_ms', r.get('kernel_ms'), 'frac', r.get('frac'), 'exec', (r.get('executed') or {}).get('valu_issue_frac'))"
done
