# occupancy A/B of the validate step (tools/kbench.py) over variant builds; usage: bash tools/gpu_ab_only.sh "<lib names>"
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for lib in $1; do
  VAMP_AMD_LIB=$PWD/mr-vamp_amd/vamp_amd/$lib.so timeout -k 10 300 python tools/kbench.py --edges 1048576 --reps 5 --tag $lib > gpurun_out/ab/$lib.json 2> gpurun_out/ab/$lib.err || { echo "kbench $lib failed"; tail -20 gpurun_out/ab/$lib.err; exit 1; }
  cat gpurun_out/ab/$lib.json
done
