# GPU tests + the prm_edges bench leg (development run)
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --workload prm_edges --steps 3 --warmup 1 > gpurun_out/bench_prm_edges.json 2> gpurun_out/bench_prm_edges.err || { echo "bench failed"; tail -30 gpurun_out/bench_prm_edges.err; exit 1; }
cat gpurun_out/bench_prm_edges.json
