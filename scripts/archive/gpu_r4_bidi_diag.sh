#!/bin/bash
# Round 4: diagnosis of the two-ended path (scripts/bidi_diag.py).  Outputs gpurun_out/r4bidi/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4bidi
mkdir -p $OUT
DIAG_CHAINS=24 DIAG_WARMUP=80 DIAG_SAMPLES=60 DIAG_SEED=33 timeout -k 10 120 python -u scripts/bidi_diag.py > $OUT/diag.log 2>&1; rc=$?
cat $OUT/diag.log
exit $rc
