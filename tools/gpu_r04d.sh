#!/bin/bash
# round-4 pass d: the composite's inter-arm bound kernels at 3 (default) vs 4 waves/EU (variant w4),
# alternating; round-set A/B of the Panda staged pass; the full-size configs[3] edge stage (bench + profile)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/r04d_pair_ab.log
for rep in 1 2; do
  for v in default w4; do
    L=mr-vamp_amd/vamp_amd/libvampgpu.so; [ $v = w4 ] && L=mr-vamp_amd/vamp_amd/libvampgpu_w4.so
    VAMP_AMD_LIB=$PWD/$L timeout -k 10 200 python bench.py --workload pair --steps 10 --warmup 2 --no-cpu > gpurun_out/r04d_pair_$v.json 2>/dev/null || { echo "pair $v failed"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r04d_pair_$v.json')); print('$v', d['roofline']['kernel_ms'])" >> gpurun_out/r04d_pair_ab.log
  done
done
cat gpurun_out/r04d_pair_ab.log
bash tools/rounds_ab.sh r04d || exit 1
timeout -k 10 600 python bench.py --workload prm_edges --vertices 2681709 --steps 3 --warmup 1 > gpurun_out/bench_r04d_prm_edges_full.json 2> gpurun_out/bench_r04d_prm_edges_full.err || { echo "prm_edges full failed"; tail -20 gpurun_out/bench_r04d_prm_edges_full.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r04d_prm_edges_full.json')); print('prm_edges_full', d['value'], d['ms_per_step'], json.dumps(d['phases'])[:600])"
bash tools/prof_r04.sh prm_edges_full
