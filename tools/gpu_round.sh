#!/bin/bash
# GPU-box passes (run through gpurun from the repo root).  One script, several modes; every GPU step runs under its
# own timeout and the script stops at the first failure (no retries).
#
#   bash tools/gpu_round.sh suite TAG [SPEC [FILE ...]]  the -m gpu suite, or the given test files (SPEC: a library
#                                                   variant, below) -> gpurun_out/TAG_gputest[_SPEC].log
#   bash tools/gpu_round.sh smoke TAG                __graft_entry__.smoke() -> gpurun_out/TAG_smoke.log
#   bash tools/gpu_round.sh bench TAG W [W ...]      bench lines with CPU baselines -> gpurun_out/TAG_bench_W.json
#   bash tools/gpu_round.sh prof W [W ...]           step profiles (tools/prof_step.sh -> gpurun_out/prof/W.json)
#   bash tools/gpu_round.sh ab TAG REPS W,W,.. SPEC SPEC ...
#                                                   alternating A/B: REPS rounds of every SPEC over the bench workloads
#                                                   W (--no-cpu), one JSON record per run -> gpurun_out/TAG_ab.log and a
#                                                   per-(workload, spec) summary; each SPEC's parity suite first
#   bash tools/gpu_round.sh final TAG                suite + smoke + every workload's bench line + every step profile
#
# W (bench workloads): validate validate_setA table_pick capt fetch_prm prm_edges prm_edges_full pair rrtc rrtc_pair
# SPEC = variant[:ENV=VAL[,ENV=VAL]]: variant "rel" is mr-vamp_amd/vamp_amd/libvampgpu.so, any other name the A/B
# build libvampgpu_<variant>.so (make -C mr-vamp_amd VARIANT=<variant> DEFS=...); ENV=VAL are run-time knobs.
# (Round 5's one-off pass scripts, tools/gpu_r05*.sh, are folded into these modes.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/mr-vamp_amd/vamp_amd
MODE=$1; shift

lib() { if [ "$1" = rel ] || [ -z "$1" ]; then echo $L/libvampgpu.so; else echo $L/libvampgpu_$1.so; fi; }
spec_env() {  # SPEC -> "VAMP_AMD_LIB=... ENV=VAL ..."
  local v=${1%%:*} e=""
  [ "$1" != "$v" ] && e=$(echo ${1#*:} | tr ',' ' ')
  echo "VAMP_AMD_LIB=$(lib $v) $e"
}
bench_args() {  # workload -> bench.py arguments
  case $1 in
    validate_setA) echo "--edge-set A" ;;
    table_pick) echo "--scene table_pick" ;;
    prm_edges_full) echo "--workload prm_edges --vertices 2681709" ;;
    rrtc_pair) echo "--workload rrtc --robot panda_pair" ;;
    *) echo "--workload $1" ;;
  esac
}
summary() {  # bench line -> one summary line on stdout
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2], '%.4g' % d['value'], d['unit'], 'ms %.4f' % d['ms_per_step'], 'frac', r.get('frac'), 'ref_work_frac', r.get('reference_work_frac'), 'parity', json.dumps(d.get('parity'))[:200])" "$1" "$2"
}
suite() {  # TAG [SPEC [FILE ...]]
  local out=gpurun_out/$1_gputest${2:+_${2%%:*}}.log spec=${2:-rel}
  shift; [ $# -gt 0 ] && shift
  local files=${*:-tests}
  env $(spec_env $spec) timeout -k 10 700 python -u -m pytest $files -m gpu -x -v --timeout 200 --timeout-method thread > $out 2>&1 || { echo "suite $spec failed: $out"; tail -30 $out; exit 1; }
  echo "suite $spec: $(tail -n 1 $out)"
}

case $MODE in
suite) suite "$@" ;;
smoke)
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$1_smoke.log 2>&1 || { tail -20 gpurun_out/$1_smoke.log; exit 1; }
  tail -n 1 gpurun_out/$1_smoke.log ;;
bench)
  T=$1; shift
  for w in "$@"; do
    steps="--steps 20 --warmup 3"; [ $w = prm_edges_full ] && steps="--steps 3 --warmup 1"
    timeout -k 10 600 python bench.py $(bench_args $w) $steps > gpurun_out/${T}_bench_$w.json 2> gpurun_out/${T}_bench_$w.err || { tail -20 gpurun_out/${T}_bench_$w.err; exit 1; }
    summary gpurun_out/${T}_bench_$w.json $w
  done ;;
prof) bash tools/prof_step.sh "$@" || exit 1 ;;
ab)
  T=$1 REPS=$2 WS=$3; shift 3
  OUT=gpurun_out/${T}_ab.log
  : > $OUT
  for s in "$@"; do  # each spec's parity first, one log per spec
    env $(spec_env $s) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fetch.py tests/test_gpu_pair.py tests/test_gpu_capt.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_parity_${s%%:*}.log 2>&1 || { echo "parity $s failed"; tail -30 gpurun_out/${T}_parity_${s%%:*}.log; exit 1; }
    echo "$s parity: $(tail -n 1 gpurun_out/${T}_parity_${s%%:*}.log)"
  done
  for r in $(seq $REPS); do
    for w in ${WS//,/ }; do
      for s in "$@"; do
        env $(spec_env $s) timeout -k 10 400 python bench.py $(bench_args $w) --steps 20 --warmup 3 --no-cpu > gpurun_out/${T}_line.json 2> gpurun_out/${T}_line.err || { echo "$w $s failed"; tail -5 gpurun_out/${T}_line.err; exit 1; }
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(json.dumps({'spec': sys.argv[2], 'workload': sys.argv[3], 'ms': d['ms_per_step'], 'kernel_ms': r.get('kernel_ms'), 'phases': {k: v for k, v in (d.get('phases') or r.get('phase_ms') or {}).items() if isinstance(v, (int, float))}}))" gpurun_out/${T}_line.json "$s" $w >> $OUT
      done
    done
  done
  python3 -c '
import sys, json, collections
r = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); r[(d["workload"], d["spec"])].append(round(d["ms"], 4))
for k, v in sorted(r.items()): print(k, v)' $OUT ;;
final)
  T=$1
  timeout -k 10 300 python -u -c "import torch; print('torch', torch.__version__, torch.cuda.is_available(), flush=True)" || exit 1
  suite $T
  bash $0 smoke $T || exit 1
  bash $0 bench $T validate validate_setA table_pick capt fetch_prm prm_edges pair rrtc rrtc_pair || exit 1
  bash tools/prof_step.sh validate validate_setA validate_table_pick capt fetch_prm pair prm_edges || exit 1 ;;
*) echo "usage: bash tools/gpu_round.sh suite|smoke|bench|prof|ab|final ..."; exit 2 ;;
esac
