#!/bin/bash
# round-4 pass l: round 1 = the most-fired environment check alone (release build): GPU suite, headline /
# set A / capt bench lines, then A/B: validate tails as one round (VAMP_AMD_ONE_ROUND=8) and mid tests in
# the configurations' bound stage (libvampgpu_cfgmid.so, kinds 0, 3, 4), capt through bench.py for both
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04l_gputest.log 2>&1 || { tail -30 gpurun_out/r04l_gputest.log; exit 1; }
tail -n 1 gpurun_out/r04l_gputest.log
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; p=d.get('parity') or {}; print(sys.argv[2], d['value'], 'ms', d['ms_per_step'], 'kernel_ms', r.get('kernel_ms'), 'mism', [v.get('mismatches') for v in p.values() if isinstance(v, dict)])" "$1" "$2"; }
for w in validate validate_setA capt; do
  a="--workload $w"; [ $w = validate_setA ] && a="--edge-set A"
  timeout -k 10 300 python bench.py $a --steps 10 --warmup 2 > gpurun_out/bench_r04l_$w.json 2> gpurun_out/bench_r04l_$w.err || { tail -20 gpurun_out/bench_r04l_$w.err; exit 1; }
  line gpurun_out/bench_r04l_$w.json $w
done
L=$PWD/mr-vamp_amd/vamp_amd
VAMP_AMD_LIB=$L/libvampgpu_cfgmid.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_staged_chains.py tests/test_gpu_capt_grid.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04l_cfgmid_parity.log 2>&1 || { tail -30 gpurun_out/r04l_cfgmid_parity.log; exit 1; }
tail -n 1 gpurun_out/r04l_cfgmid_parity.log
: > gpurun_out/r04l_ab.log
for r in 1 2; do
  timeout -k 10 200 python tools/kbench.py --tag default >> gpurun_out/r04l_ab.log 2>/dev/null || exit 1
  VAMP_AMD_ONE_ROUND=8 timeout -k 10 200 python tools/kbench.py --tag tail1round >> gpurun_out/r04l_ab.log 2>/dev/null || exit 1
  VAMP_AMD_LIB=$L/libvampgpu_cfgmid.so timeout -k 10 200 python tools/kbench.py --tag cfgmid >> gpurun_out/r04l_ab.log 2>/dev/null || exit 1
  for v in default cfgmid; do
    lib=$L/libvampgpu.so; [ $v = cfgmid ] && lib=$L/libvampgpu_cfgmid.so
    VAMP_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload capt --steps 10 --warmup 2 --no-cpu > gpurun_out/capt_ab.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/capt_ab.json')); print(json.dumps({'tag': '$v', 'kernel': 'capt', 'ms': d['ms_per_step']}))" >> gpurun_out/r04l_ab.log
  done
done
grep -v amdgpu.ids gpurun_out/r04l_ab.log | python3 -c '
import sys, json, collections
r = collections.defaultdict(list)
for l in sys.stdin:
    d = json.loads(l); r[(d["kernel"], d["tag"])].append(d["ms"])
for k, v in sorted(r.items()): print(k, ["%.3f" % x for x in v])'
