#!/bin/bash
# Round 4: the whole GPU test suite on the current tree.  Outputs gpurun_out/r4suite/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4suite
mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=15 > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -25 $OUT/pytest_gpu.log
exit $rc
