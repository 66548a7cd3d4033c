#!/bin/bash
# Round 5: the whole GPU test suite on the current tree, then smoke().  gpurun_out/r5suite/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5suite
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=15 > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -25 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?
cat $OUT/smoke.log | tail -3
exit $rc
