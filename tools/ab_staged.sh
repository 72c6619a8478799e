set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
VAMP_AMD_STAGED=0 timeout -k 10 300 python tools/kbench.py --edges 1048576 --reps 5 --tag mono || exit 1
VAMP_AMD_STAGED=1 timeout -k 10 300 python tools/kbench.py --edges 1048576 --reps 5 --tag staged_auto || exit 1
VAMP_AMD_STAGED=1 VAMP_AMD_ROUNDS=0x118,0xffdf7ee7,0x208000 timeout -k 10 300 python tools/kbench.py --edges 1048576 --reps 5 --tag staged_3r || exit 1
