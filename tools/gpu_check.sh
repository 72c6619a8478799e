#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-all}
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
lscpu > gpurun_out/lscpu.txt 2>&1 || true
if [ "$STEP" = "all" ] || [ "$STEP" = "test" ]; then
  timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "bench" ]; then
  timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "prof" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*stats*" | head
fi
echo done
