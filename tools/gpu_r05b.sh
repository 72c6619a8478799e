set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_multi.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r05b_multi.log 2>&1; rc=$?
grep -E "PASS|FAIL|SKIP|^E " gpurun_out/r05b_multi.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05b_gputest.log 2>&1 || { tail -30 gpurun_out/r05b_gputest.log; exit 1; }
tail -2 gpurun_out/r05b_gputest.log
for w in fetch_prm prm_edges; do
  timeout -k 10 400 python bench.py --workload $w --steps 10 --warmup 2 > gpurun_out/r05b_bench_$w.json 2> gpurun_out/r05b_bench_$w.err || { tail -20 gpurun_out/r05b_bench_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['unit'], 'ms', d['ms_per_step'], 'frac', r.get('frac'), 'parity', d.get('parity'))" gpurun_out/r05b_bench_$w.json $w
done
