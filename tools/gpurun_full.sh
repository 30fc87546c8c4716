#!/bin/bash
# full GPU regression: every -m gpu test, then smoke() (skipped after a crash or timeout)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
T=${TAG:-full}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_pytest.log 2>&1
rc=$?
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
exit $rc
