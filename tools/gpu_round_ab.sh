set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for lib in libvampgpu libvampgpu_c6 libvampgpu_c5 libvampgpu_b6c6; do
  VAMP_AMD_LIB=$PWD/mr-vamp_amd/vamp_amd/$lib.so timeout -k 10 300 python tools/kbench.py --edges 1048576 --reps 5 --tag $lib > gpurun_out/ab/$lib.json 2> gpurun_out/ab/$lib.err || { echo "kbench $lib failed"; tail -20 gpurun_out/ab/$lib.err; exit 1; }
  cat gpurun_out/ab/$lib.json
done
