#!/bin/bash
# round-4 pass j: the GPU suite on the release build (grid-header readback test included), the CAPT bench
# and profile after the layout fix, then the mid-level sphere filter variant: parity suites and an A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04j_gputest.log 2>&1 || { tail -30 gpurun_out/r04j_gputest.log; exit 1; }
tail -1 gpurun_out/r04j_gputest.log
timeout -k 10 300 python bench.py --workload capt --steps 10 --warmup 2 > gpurun_out/bench_r04j_capt.json 2> gpurun_out/bench_r04j_capt.err || { tail -20 gpurun_out/bench_r04j_capt.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r04j_capt.json')); r=d['roofline']; print('capt', d['value'], 'ms', d['ms_per_step'], 'kernel_ms', r.get('kernel_ms'))"
bash tools/prof_r04.sh capt || exit 1
L=$PWD/mr-vamp_amd/vamp_amd/libvampgpu_mid.so
VAMP_AMD_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_staged_chains.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04j_mid_parity.log 2>&1 || { tail -30 gpurun_out/r04j_mid_parity.log; exit 1; }
tail -1 gpurun_out/r04j_mid_parity.log
timeout -k 10 200 python tools/kbench.py --tag default > gpurun_out/r04j_ab.log 2>&1 || { tail -20 gpurun_out/r04j_ab.log; exit 1; }
VAMP_AMD_LIB=$L timeout -k 10 200 python tools/kbench.py --tag mid >> gpurun_out/r04j_ab.log 2>&1 || { tail -20 gpurun_out/r04j_ab.log; exit 1; }
timeout -k 10 200 python tools/kbench.py --tag default2 >> gpurun_out/r04j_ab.log 2>&1 || { tail -20 gpurun_out/r04j_ab.log; exit 1; }
cat gpurun_out/r04j_ab.log
