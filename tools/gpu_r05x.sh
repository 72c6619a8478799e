#!/bin/bash
# round-5 pass x: the edge-stage lines with the Roadmap left in HBM (its host copy timed beside value as
# phases.pcie_inclusive_*): 100k and 2.68M vertices, with their CPU baselines and graph parity
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload prm_edges --steps 20 --warmup 3 > gpurun_out/r05_bench_prm_edges.json 2> gpurun_out/r05_bench_prm_edges.err || { tail -20 gpurun_out/r05_bench_prm_edges.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05_bench_prm_edges.json')); p=d['phases']; print('prm_edges', d['value'], 'ms', round(d['ms_per_step'], 3), 'pcie', round(p['pcie_inclusive_ms_per_step'], 3), 'parity', json.dumps(d.get('parity'))[:200])"
timeout -k 10 600 python bench.py --workload prm_edges --vertices 2681709 --steps 3 --warmup 1 > gpurun_out/r05_bench_prm_edges_full.json 2> gpurun_out/r05_bench_prm_edges_full.err || { tail -20 gpurun_out/r05_bench_prm_edges_full.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05_bench_prm_edges_full.json')); print('prm_edges_full', d['value'], 'ms', round(d['ms_per_step'], 2), 'phases', {k: round(v, 1) for k, v in d['phases'].items() if 'ms' in k}, 'parity', json.dumps(d.get('parity'))[:300])"
