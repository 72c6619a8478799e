#!/bin/bash
# CAPT LDS-staging A/B on the GPU box (development): parity tests of the point-cloud paths, then
# tools/kbench_capt.py for each library variant.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_capt.py -q --timeout 120 --timeout-method thread \
    > gpurun_out/ab_capt_tests.log 2>&1 || exit 1
for v in "" _lds0 _lds10 _lds13; do
    VAMP_AMD_LIB=mr-vamp_amd/vamp_amd/libvampgpu$v.so timeout -k 10 120 python -u tools/kbench_capt.py \
        >> gpurun_out/ab_capt.log 2>&1 || exit 2
done
