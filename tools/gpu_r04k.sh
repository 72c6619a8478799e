#!/bin/bash
# round-4 pass k: mid-sphere tests in the validate tails' bound stage (VGPU_PANDA_MID_KINDS): the GPU suite
# on the release build (tails: 0x18), then an alternating A/B against no mid kinds and head + tails
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04k_gputest.log 2>&1 || { tail -30 gpurun_out/r04k_gputest.log; exit 1; }
tail -n 1 gpurun_out/r04k_gputest.log
L=$PWD/mr-vamp_amd/vamp_amd
VAMP_AMD_LIB=$L/libvampgpu_headmid.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_staged_chains.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04k_headmid_parity.log 2>&1 || { tail -30 gpurun_out/r04k_headmid_parity.log; exit 1; }
tail -n 1 gpurun_out/r04k_headmid_parity.log
: > gpurun_out/r04k_ab.log
for r in 1 2; do
  for v in tails nomid headmid; do
    if [ $v = tails ]; then lib=$L/libvampgpu.so; else lib=$L/libvampgpu_$v.so; fi
    VAMP_AMD_LIB=$lib timeout -k 10 200 python tools/kbench.py --tag $v >> gpurun_out/r04k_ab.log 2>/dev/null || { echo "kbench $v failed"; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/r04k_ab.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_r04k_validate.json 2> gpurun_out/bench_r04k_validate.err || { tail -20 gpurun_out/bench_r04k_validate.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r04k_validate.json')); r=d['roofline']; print('validate', d['value'], 'ms', d['ms_per_step'], 'kernel_ms', r.get('kernel_ms'), 'parity', d.get('parity'))"
# rounds led by check 8 alone (the link-5 environment check: fires for ~every set A head group, 97 % confirm)
SETS="default 0x100,0x18,0xfffffee7 0x100,0xfffffeff 0x100,0x18,0x80430800,0x7fbcf6e0" timeout -k 10 600 bash tools/rounds_ab.sh r04k || exit 1
