set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r06zu bash tools/gpu_steps.sh gpu smoke bench c3 || exit $?
timeout -k 10 300 python tools/c3_host_profile.py > gpurun_out/r06zu_c3host.txt 2>&1
head -3 gpurun_out/r06zu_c3host.txt
