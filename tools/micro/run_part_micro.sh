# usage: bash tools/micro/run_part_micro.sh [rows] [reps] -- build and run the C3 partition micro-benchmark on the GPU box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/micro
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -I bqueryd_amd/csrc -I include tools/micro/part_micro.hip -o gpurun_out/micro/part_micro || exit $?
timeout -k 10 120 gpurun_out/micro/part_micro "$@"
