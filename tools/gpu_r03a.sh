#!/bin/bash
# Round-3 GPU pass: the new GPU tests first (configs[0] on the HIP path, table_pick GPU legs, the
# 1.3M-vertex kNN index, the device-built cloud realised from its host twin, the 2^32-block guard),
# then the whole -m gpu suite, then the validate variants of SURVEY §8(d) config 2.
# usage: bash tools/gpu_r03a.sh TAG
TAG=${1:-r03a}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rrtc.py tests/test_gpu_capt_build.py tests/test_gpu_parity.py \
    "tests/test_gpu_roadmap.py::test_knn_index_equals_brute_force_large" -v -s --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_newtests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_gputest.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench_validate.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --edge-set A --no-fk-leg > gpurun_out/${TAG}_bench_setA.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --base 220 --no-fk-leg > gpurun_out/${TAG}_bench_b220.log 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --scene table_pick --no-fk-leg > gpurun_out/${TAG}_bench_tablepick.log 2>&1 || exit 6
