set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r06zs bash tools/gpu_steps.sh gpu smoke bench prof || exit $?
