#!/bin/bash
# round-5 pass q: the CAPT cell grid in 4 x 4 x 4 bricks (VGPU_CAPT_BRICK=1) vs x-fastest rows: the -m gpu suite
# both ways, then the CAPT step alternating, and each layout's grid build under a kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05q_gputest.log 2>&1 || { tail -30 gpurun_out/r05q_gputest.log; exit 1; }
tail -n 1 gpurun_out/r05q_gputest.log
VGPU_CAPT_BRICK=1 timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05q_gputest_brick.log 2>&1 || { tail -30 gpurun_out/r05q_gputest_brick.log; exit 1; }
echo "brick: $(tail -n 1 gpurun_out/r05q_gputest_brick.log)"
: > gpurun_out/r05q_capt.log
for r in 1 2 3; do
  for b in 0 1; do
    VGPU_CAPT_BRICK=$b timeout -k 10 300 python bench.py --workload capt --steps 20 --warmup 3 --no-cpu > gpurun_out/r05q_line.json 2>/dev/null || { echo "capt brick=$b failed"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r05q_line.json')); print(json.dumps({'brick': $b, 'ms': d['ms_per_step'], 'kernel_ms': d['roofline'].get('kernel_ms'), 'raw': d.get('raw_queries', {}).get('ms')}))" | tee -a gpurun_out/r05q_capt.log
  done
done
for b in 0 1; do
  VGPU_CAPT_BRICK=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05q_capt_b$b -o capt --output-format csv -- python3 bench.py --workload capt --steps 5 --warmup 1 --no-cpu > gpurun_out/r05q_capt_prof_b$b.log 2>&1 || { echo "capt prof $b failed"; tail -5 gpurun_out/r05q_capt_prof_b$b.log; exit 1; }
  find gpurun_out/r05q_capt_b$b -name "*kernel_stats.csv" -exec grep -h "capt_grid_kernel\|children_kernel<vgpu::PandaR, vgpu::SrcConfigsT<vgpu::PandaR>, true, 0>\|bound_kernel<vgpu::PandaR, vgpu::SrcConfigsT<vgpu::PandaR>, true>" {} \; | cut -c1-40,150-260
done
