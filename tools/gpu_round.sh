#!/bin/bash
# One measurement pass on the GPU box (gpurun): the -m gpu suite, every workload's bench line
# (gpurun_out/bench_<tag>_<workload>.json), then a profile of every workload's step (tools/prof_step.sh:
# kernel trace + SQ/TCC PMC -> gpurun_out/prof/).   usage: bash tools/gpu_round.sh TAG [--debug]
# --debug: the suite on the bounds-checked build (make -C mr-vamp_amd DEBUG=1) first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-run}
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import torch; print('torch', torch.__version__, torch.cuda.is_available(), flush=True)" || exit 1
if [ "$2" = "--debug" ]; then
  VAMP_AMD_LIB=$PWD/mr-vamp_amd/vamp_amd/libvampgpu_debug.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_gputest_debug.log 2>&1 || { tail -30 gpurun_out/${T}_gputest_debug.log; exit 1; }
  tail -n 1 gpurun_out/${T}_gputest_debug.log
fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1 || { tail -30 gpurun_out/${T}_gputest.log; exit 1; }
tail -n 1 gpurun_out/${T}_gputest.log
for w in validate validate_setA capt fetch_prm prm_edges pair rrtc; do
  a="--workload $w"; [ $w = validate_setA ] && a="--edge-set A"
  timeout -k 10 300 python bench.py $a --steps 10 --warmup 2 > gpurun_out/bench_${T}_$w.json 2> gpurun_out/bench_${T}_$w.err || { tail -20 gpurun_out/bench_${T}_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2], d['value'], d['unit'], 'ms', d['ms_per_step'], 'kernel_ms', r.get('kernel_ms'))" gpurun_out/bench_${T}_$w.json $w
done
bash tools/prof_step.sh validate validate_setA capt fetch_prm pair prm_edges || exit 1
