#!/bin/bash
# round-4 pass m: the lead pass (check 8 monolithic before the chained bound stage; Panda validate heads) and
# validate tails as one round: GPU suite, A/B of the lead kinds (VAMP_AMD_LEAD: 0 none, 4 heads, 5 heads +
# configurations), bench lines, then fresh profiles of validate and set A for the executed block
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04m_gputest.log 2>&1 || { tail -30 gpurun_out/r04m_gputest.log; exit 1; }
tail -n 1 gpurun_out/r04m_gputest.log
VAMP_AMD_LEAD=5 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_staged_chains.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04m_lead5_parity.log 2>&1 || { tail -30 gpurun_out/r04m_lead5_parity.log; exit 1; }
tail -n 1 gpurun_out/r04m_lead5_parity.log
: > gpurun_out/r04m_ab.log
for r in 1 2; do
  for k in 4 0 5; do
    VAMP_AMD_LEAD=$k timeout -k 10 200 python tools/kbench.py --tag lead$k >> gpurun_out/r04m_ab.log 2>/dev/null || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/r04m_ab.log | python3 -c '
import sys, json, collections
r = collections.defaultdict(list)
for l in sys.stdin:
    d = json.loads(l); r[(d["kernel"], d["tag"])].append(d["ms"])
for k, v in sorted(r.items()): print(k, ["%.3f" % x for x in v])'
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; p=d.get('parity') or {}; print(sys.argv[2], d['value'], 'ms', d['ms_per_step'], 'kernel_ms', r.get('kernel_ms'), 'mism', [v.get('mismatches') for v in p.values() if isinstance(v, dict)])" "$1" "$2"; }
for w in validate validate_setA capt; do
  a="--workload $w"; [ $w = validate_setA ] && a="--edge-set A"
  timeout -k 10 300 python bench.py $a --steps 10 --warmup 2 > gpurun_out/bench_r04m_$w.json 2> gpurun_out/bench_r04m_$w.err || { tail -20 gpurun_out/bench_r04m_$w.err; exit 1; }
  line gpurun_out/bench_r04m_$w.json $w
done
bash tools/prof_r04.sh validate validate_setA || exit 1
# variant q: the queue kernel's per-block check bases in LDS, and the CAPT grid build's leaf-box pruning
Q=$PWD/mr-vamp_amd/vamp_amd/libvampgpu_q.so
VAMP_AMD_LIB=$Q timeout -k 10 400 python -u -m pytest tests/test_gpu_capt_grid.py tests/test_gpu_parity.py tests/test_gpu_staged_chains.py tests/test_gpu_env_incremental.py tests/test_gpu_roadmap.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04m_q_parity.log 2>&1 || { tail -30 gpurun_out/r04m_q_parity.log; exit 1; }
tail -n 1 gpurun_out/r04m_q_parity.log
: > gpurun_out/r04m_q_ab.log
for r in 1 2; do
  for v in rel q; do
    lib=$PWD/mr-vamp_amd/vamp_amd/libvampgpu.so; [ $v = q ] && lib=$Q
    VAMP_AMD_LIB=$lib timeout -k 10 200 python tools/kbench.py --tag $v >> gpurun_out/r04m_q_ab.log 2>/dev/null || exit 1
    for w in fetch_prm capt; do
      VAMP_AMD_LIB=$lib timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu > gpurun_out/q_ab.json 2>/dev/null || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/q_ab.json')); print(json.dumps({'tag': '$v', 'kernel': '$w', 'ms': d['ms_per_step'], 'kernel_ms': d['roofline'].get('kernel_ms'), 'upload_ms': (d.get('environment_upload_ms') or {}).get('ms')}))" >> gpurun_out/r04m_q_ab.log
    done
  done
done
grep -v amdgpu.ids gpurun_out/r04m_q_ab.log | python3 -c '
import sys, json, collections
r = collections.defaultdict(list)
for l in sys.stdin:
    d = json.loads(l); r[(d["kernel"], d["tag"])].append("%.3f/%s" % (d["ms"], d.get("upload_ms") and "%.2f" % d["upload_ms"]))
for k, v in sorted(r.items()): print(k, v)'
mkdir -p gpurun_out/qtrace
VAMP_AMD_LIB=$Q timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/qtrace/raw -o trace --output-format csv -- python3 tools/pmc_drive.py run --workload capt --calls 2 > gpurun_out/qtrace/trace.log 2>&1 || { tail -20 gpurun_out/qtrace/trace.log; exit 1; }
cp $(find gpurun_out/qtrace/raw -name "*kernel_stats.csv" | head -1) gpurun_out/qtrace/capt_q_kernel_stats.csv && rm -rf gpurun_out/qtrace/raw
grep -i "capt_grid" gpurun_out/qtrace/capt_q_kernel_stats.csv | cut -c1-200
