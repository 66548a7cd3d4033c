#!/bin/bash
# Round 4: per-chain diagnosis of the hard-geometry R-hat at seed 1019 (1.0146) against 1001 (1.0084).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4hd
mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/hard_diag.py 1019 > $OUT/diag_1019.json 2> $OUT/diag.err || { tail -20 $OUT/diag.err; exit 1; }
timeout -k 10 300 python3 -u scripts/hard_diag.py 1001 > $OUT/diag_1001.json 2>> $OUT/diag.err || { tail -20 $OUT/diag.err; exit 1; }
echo done
