#!/bin/bash
# Round 5: config 5 across this round's commits on one box (each tree's own bench.py and
# library), interleaved twice.  gpurun_out/r5bisect/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5bisect
mkdir -p $OUT
for r in 1 2; do
  for d in ablib/wt_r4 ablib/wt_b2bd664 ablib/wt_9be2c73 ablib/wt_33ebe85 ablib/wt_a5fe83c .; do
    (cd $d && timeout -k 10 200 python3 bench.py --config ${CFG:-5} --steps 2 --warmup 1 --no-cpu \
      2>>$GRAFT_REPO_ROOT/$OUT/stderr.log) > $OUT/ab.json || exit 1
    python3 -c "import json;d=json.load(open('$OUT/ab.json'));print('$d', d['value'], d['roofline']['kernel_ms'])" | tee -a $OUT/ab.txt
  done
done
