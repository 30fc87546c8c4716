set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r06zr bash tools/gpu_steps.sh profc4 || exit $?
cat gpurun_out/r06zr_profc4_shapes.txt | head -40
