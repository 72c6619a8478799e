#!/bin/bash
# round-5 pass u2 (final build): the edge-stage step profiles, then every workload's bench line with its CPU
# baseline (gpurun_out/r05_bench_<w>.json; the prm_edges lines read the profiles just taken), the full-size edge
# stage, and the rocprofv3 kernel-trace summary of the default bench command
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/prof_step.sh prm_edges prm_edges_full || exit 1
for w in prm_edges prm_edges_full; do cp gpurun_out/prof/$w.json profiles/r05_prof_$w.json; done
for w in validate validate_setA table_pick capt fetch_prm prm_edges pair rrtc; do
  a="--workload $w"; [ $w = validate_setA ] && a="--edge-set A"; [ $w = table_pick ] && a="--scene table_pick"
  timeout -k 10 300 python bench.py $a --steps 20 --warmup 3 > gpurun_out/r05_bench_$w.json 2> gpurun_out/r05_bench_$w.err || { tail -20 gpurun_out/r05_bench_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2], d['value'], d['unit'], 'ms', round(d['ms_per_step'], 4), 'frac', r.get('frac'), 'parity', json.dumps(d.get('parity'))[:160])" gpurun_out/r05_bench_$w.json $w
done
timeout -k 10 600 python bench.py --workload prm_edges --vertices 2681709 --steps 3 --warmup 1 > gpurun_out/r05_bench_prm_edges_full.json 2> gpurun_out/r05_bench_prm_edges_full.err || { tail -20 gpurun_out/r05_bench_prm_edges_full.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05_bench_prm_edges_full.json')); print('prm_edges_full', d['value'], d['unit'], 'ms', round(d['ms_per_step'], 2), 'phases', {k: round(v, 1) for k, v in d['phases'].items() if k.endswith('_ms')}, 'parity', json.dumps(d.get('parity'))[:300])"
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_benchprof -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/r05_benchprof.log 2>&1 || { tail -10 gpurun_out/r05_benchprof.log; exit 1; }
find gpurun_out/r05_benchprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r05_bench_kernel_stats.csv \;
head -5 gpurun_out/r05_bench_kernel_stats.csv | cut -c1-160
