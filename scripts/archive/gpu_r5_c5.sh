#!/bin/bash
# Round 5: same-box A/B of config 5 (and 2): HEAD, the sweep-contraction variant, and the
# round-4 final tree (ablib/wt_r4, its own bench.py), interleaved.  gpurun_out/r5c5/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5c5
mkdir -p $OUT
run() {   # label, dir, config, env...
  local l=$1; local d=$2; local c=$3; shift; shift; shift
  (cd $d && env "$@" timeout -k 10 200 python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu \
    2>>$GRAFT_REPO_ROOT/$OUT/stderr.log) > $OUT/ab.json || exit 1
  python3 -c "import json;d=json.load(open('$OUT/ab.json'));print('$l config $c', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" | tee -a $OUT/ab.txt
}
for r in 1 2 3; do
  for c in 5 2; do
    run head . $c FITOCT_X=0
    run sweepfast . $c FITOCT_LIB_PATH=$GRAFT_REPO_ROOT/ablib/lib_sweepfast.so
    run r4 ablib/wt_r4 $c FITOCT_X=0
  done
done
