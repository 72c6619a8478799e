#!/bin/bash
# round-5 pass n (final build: composite tails with mid spheres, roadmap offsets from the sorted keys): the -m gpu
# suite (and on the bounds-checked build when present), the step profiles of the workloads whose kernels changed
# since pass k (pair, prm_edges, prm_edges_full) -- copied into profiles/ here so the bench lines that follow read
# them -- and those bench lines with their CPU baselines and graph parity
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/mr-vamp_amd/vamp_amd
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r05n_gputest.log 2>&1 || { tail -30 gpurun_out/r05n_gputest.log; exit 1; }
tail -n 1 gpurun_out/r05n_gputest.log
if [ -f $L/libvampgpu_debug.so ]; then
  VAMP_AMD_LIB=$L/libvampgpu_debug.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05n_gputest_debug.log 2>&1 || { tail -30 gpurun_out/r05n_gputest_debug.log; exit 1; }
  echo "debug: $(tail -n 1 gpurun_out/r05n_gputest_debug.log)"
fi
bash tools/prof_step.sh pair prm_edges prm_edges_full || exit 1
for w in pair prm_edges prm_edges_full; do cp gpurun_out/prof/$w.json profiles/r05_prof_$w.json; done
for w in pair prm_edges; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 > gpurun_out/r05_bench_$w.json 2> gpurun_out/r05_bench_$w.err || { tail -20 gpurun_out/r05_bench_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2], d['value'], d['unit'], 'ms', round(d['ms_per_step'], 4), 'frac', r.get('frac'), 'parity', json.dumps(d.get('parity'))[:160])" gpurun_out/r05_bench_$w.json $w
done
timeout -k 10 600 python bench.py --workload prm_edges --vertices 2681709 --steps 3 --warmup 1 > gpurun_out/r05_bench_prm_edges_full.json 2> gpurun_out/r05_bench_prm_edges_full.err || { tail -20 gpurun_out/r05_bench_prm_edges_full.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05_bench_prm_edges_full.json')); print('prm_edges_full', d['value'], d['unit'], 'ms', round(d['ms_per_step'], 2), 'phases', {k: round(v, 1) for k, v in d['phases'].items() if k.endswith('_ms')}, 'parity', json.dumps(d.get('parity'))[:200])"
