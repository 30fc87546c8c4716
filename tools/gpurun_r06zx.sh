set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r06zx bash tools/gpu_steps.sh gpu smoke bench || exit $?
