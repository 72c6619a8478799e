#!/bin/bash
# round-4 pass n: the release build with the lead pass and the queue change: GPU suite, Fetch hit statistics
# (libvampgpu_hs.so), every workload's bench line, then fresh profiles of every workload's step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04n_gputest.log 2>&1 || { tail -30 gpurun_out/r04n_gputest.log; exit 1; }
tail -n 1 gpurun_out/r04n_gputest.log
VAMP_AMD_LIB=$PWD/mr-vamp_amd/vamp_amd/libvampgpu_hs.so timeout -k 10 200 python tools/hitstats.py --fetch > gpurun_out/r04n_hitstats_fetch.json 2> gpurun_out/r04n_hitstats_fetch.err || { tail -20 gpurun_out/r04n_hitstats_fetch.err; exit 1; }
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; p=d.get('parity') or {}; print(sys.argv[2], d['value'], 'ms', d['ms_per_step'], 'kernel_ms', r.get('kernel_ms'), 'mism', [v.get('mismatches') for v in p.values() if isinstance(v, dict)] if isinstance(p, dict) else p)" "$1" "$2"; }
for w in validate validate_setA capt fetch_prm prm_edges pair rrtc; do
  a="--workload $w"; [ $w = validate_setA ] && a="--edge-set A"
  timeout -k 10 300 python bench.py $a --steps 10 --warmup 2 > gpurun_out/bench_r04n_$w.json 2> gpurun_out/bench_r04n_$w.err || { tail -20 gpurun_out/bench_r04n_$w.err; exit 1; }
  line gpurun_out/bench_r04n_$w.json $w
done
bash tools/prof_r04.sh validate validate_setA capt fetch_prm pair prm_edges || exit 1
