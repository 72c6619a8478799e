#!/bin/bash
# round-5 pass u1 (final build: CAPT grid in bricks + split planes): the -m gpu suite, smoke(), and the step
# profiles of the Panda / composite / Fetch vertex workloads (tools/prof_step.sh -> gpurun_out/prof/<w>.json)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r05u_gputest.log 2>&1 || { tail -30 gpurun_out/r05u_gputest.log; exit 1; }
tail -n 1 gpurun_out/r05u_gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05u_smoke.log 2>&1 || { tail -20 gpurun_out/r05u_smoke.log; exit 1; }
tail -n 1 gpurun_out/r05u_smoke.log
bash tools/prof_step.sh validate validate_setA pair fetch_prm || exit 1
