#!/bin/bash
# Round-3 pass d: chained staged passes (composite, Baxter), wrist gate, held children, multi-device /
# RCCL C entry points; then the whole -m gpu suite and the validate / pair benches.
TAG=${1:-r03d}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_staged_chains.py tests/test_multi.py tests/test_gpu_pair.py \
    tests/test_gpu_robots.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_newtests.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gputest.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench_validate.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --workload pair > gpurun_out/${TAG}_bench_pair.log 2>&1 || exit 4
timeout -k 10 300 python -u tools/kbench.py --edges 1048576 --reps 5 > gpurun_out/${TAG}_kbench.log 2>&1 || exit 5
