# kernel-trace stats of tools/kbench.py (validate set B/A, fkcc, sphere_fk) for one library
# usage: bash tools/gpu_kprof.sh <lib name> <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VAMP_AMD_LIB=$PWD/mr-vamp_amd/vamp_amd/$1.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof_$2 -o kb --output-format csv -- python3 tools/kbench.py --edges 1048576 --reps 5 --tag $2 > gpurun_out/kprof_$2.log 2>&1 || { echo "kprof $2 failed"; tail -20 gpurun_out/kprof_$2.log; exit 1; }
