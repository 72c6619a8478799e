#!/bin/bash
# One GPU-box pass (run through gpurun from the repo root): GPU parity tests, the CPU-rake tests on
# the box's host (its own rsqrt table), and the bench legs.  Every step is time-limited; the chain
# stops at the first failure.   usage: bash tools/gpu_check.sh TAG [workloads...]
TAG=${1:-r02}
shift
WL=${*:-validate capt pair fetch_prm}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_gputest.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_cpu_rake.py tests/test_c_abi.py -q --timeout 200 \
    > gpurun_out/${TAG}_cputest_box.log 2>&1 || exit 2
for w in $WL; do
    timeout -k 10 300 python -u bench.py --workload $w > gpurun_out/${TAG}_bench_$w.log 2>&1 || exit 3
done
