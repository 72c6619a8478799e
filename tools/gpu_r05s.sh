#!/bin/bash
# round-5 pass s: CAPT cell bounds and start nodes in separate planes (VGPU_CAPT_SPLIT, default 1; bricks on):
# the -m gpu suite, capt step split=1 (default) vs split=0, the grid build's kernel trace, then the capt step
# profile (tools/prof_step.sh) and the capt bench line with its CPU baseline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05s_gputest.log 2>&1 || { tail -30 gpurun_out/r05s_gputest.log; exit 1; }
tail -n 1 gpurun_out/r05s_gputest.log
: > gpurun_out/r05s_capt.log
for r in 1 2; do
  for b in 1 0; do
    VGPU_CAPT_SPLIT=$b timeout -k 10 300 python bench.py --workload capt --steps 20 --warmup 3 --no-cpu > gpurun_out/r05s_line.json 2>/dev/null || { echo "capt split=$b failed"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r05s_line.json')); u=d.get('environment_upload_ms', {}).get('ms'); print(json.dumps({'split': $b, 'ms': d['ms_per_step'], 'upload_ms': u}))" | tee -a gpurun_out/r05s_capt.log
  done
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05s_capt_prof -o capt --output-format csv -- python3 bench.py --workload capt --steps 5 --warmup 1 --no-cpu > gpurun_out/r05s_capt_prof.log 2>&1 || { echo "capt prof failed"; tail -5 gpurun_out/r05s_capt_prof.log; exit 1; }
find gpurun_out/r05s_capt_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r05s_capt_kernel_stats.csv \;
grep -h "capt_grid_kernel" gpurun_out/r05s_capt_kernel_stats.csv | cut -c1-200
bash tools/prof_step.sh capt || exit 1
timeout -k 10 300 python bench.py --workload capt --steps 20 --warmup 3 > gpurun_out/r05_bench_capt.json 2> gpurun_out/r05_bench_capt.err || { tail -20 gpurun_out/r05_bench_capt.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05_bench_capt.json')); r=d.get('roofline') or {}; print('capt', d['value'], d['unit'], 'ms', round(d['ms_per_step'], 4), 'frac', r.get('frac'), 'parity', json.dumps(d.get('parity'))[:160])"
