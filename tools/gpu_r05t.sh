#!/bin/bash
# round-5 pass t: the grid build's distance loop without the finiteness test (abs modifiers, max3):
# the CAPT GPU tests, the capt step, the grid build's kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "capt or pointcloud or env_incremental" --timeout 200 --timeout-method thread > gpurun_out/r05t_gputest.log 2>&1 || { tail -30 gpurun_out/r05t_gputest.log; exit 1; }
tail -n 1 gpurun_out/r05t_gputest.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --workload capt --steps 20 --warmup 3 --no-cpu > gpurun_out/r05t_line.json 2>/dev/null || { echo "capt failed"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05t_line.json')); u=d.get('environment_upload_ms', {}).get('ms'); print(json.dumps({'ms': d['ms_per_step'], 'upload_ms': u}))" | tee -a gpurun_out/r05t_capt.log
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05t_capt_prof -o capt --output-format csv -- python3 bench.py --workload capt --steps 5 --warmup 1 --no-cpu > gpurun_out/r05t_capt_prof.log 2>&1 || { echo "capt prof failed"; tail -5 gpurun_out/r05t_capt_prof.log; exit 1; }
find gpurun_out/r05t_capt_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r05t_capt_kernel_stats.csv \;
grep -h "capt_grid_kernel" gpurun_out/r05t_capt_kernel_stats.csv | cut -c1-200
