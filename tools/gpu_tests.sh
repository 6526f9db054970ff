#!/bin/bash
# Whole -m gpu suite in one process, then the smoke entry. Usage: bash tools/gpu_tests.sh TAG
set -o pipefail
TAG=${1:-tests}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > gpurun_out/$TAG/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$TAG/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/$TAG/smoke.log
