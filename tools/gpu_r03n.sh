#!/bin/bash
# Round-3 pass n: the Panda bound kernels with SLP packing (own translation unit): the whole -m gpu suite,
# the headline bench + kbench, the capt line, and the configs[3] edge stage at full size with its phase split.
TAG=${1:-r03n}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench_validate.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/kbench.py --edges 1048576 --reps 5 > gpurun_out/${TAG}_kbench.log 2>&1 || exit 2
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gputest.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --workload capt > gpurun_out/${TAG}_bench_capt.log 2>&1 || exit 4
timeout -k 10 600 python -u bench.py --workload prm_edges --vertices 2681709 --steps 2 --warmup 1 \
    > gpurun_out/${TAG}_bench_prm_edges_full.log 2>&1 || exit 5
