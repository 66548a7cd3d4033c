#!/bin/bash
# Round 4: per-chain diagnosis of the hard-geometry R-hat at seed 1019 (1.0146) against 1001 (1.0084).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4hd
mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/hard_diag.py 1019 > $OUT/diag_1019.json 2> $OUT/diag.err || { tail -20 $OUT/diag.err; exit 1; }
timeout -k 10 300 python3 -u scripts/hard_diag.py 1001 > $OUT/diag_1001.json 2>> $OUT/diag.err || { tail -20 $OUT/diag.err; exit 1; }

timeout -k 10 500 python -u -m pytest tests/test_gpu_funnel.py tests/test_rshim_driver.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_funnel.log 2>&1 || { tail -40 $OUT/pytest_funnel.log; exit 1; }
tail -5 $OUT/pytest_funnel.log
