#!/bin/bash
# Round 5: same-box A/B of sweep-arithmetic variants (ablib/lib_v1: no hand-fused sums,
# sweep contracted per expression; lib_v2: also the old fast contraction; HEAD: hand-fused
# sums) against the round-4 tree (ablib/wt_r4) and the last tree before the tail work
# (ablib/wt_33ebe85), configs 5, 2 and a short config 3.  gpurun_out/r5var/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5var
mkdir -p $OUT
run() {   # label, dir, config, iters, env...
  local l=$1; local d=$2; local c=$3; local it=$4; shift; shift; shift; shift
  (cd $d && env "$@" timeout -k 10 200 python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu --no-hard $it \
    2>>$GRAFT_REPO_ROOT/$OUT/stderr.log) > $OUT/ab.json || exit 1
  python3 -c "import json;d=json.load(open('$OUT/ab.json'));print('$l config $c', d['value'], d['roofline']['kernel_ms'])" | tee -a $OUT/ab.txt
}
for r in 1 2; do
  for c in 5 2 3; do
    it=""; [ $c = 3 ] && it="--iters 150,150"
    run r4 ablib/wt_r4 $c "$it" FITOCT_X=0
    run head-on-u . $c "$it" FITOCT_X=0
    run on-u-acc . $c "$it" FITOCT_LIB_PATH=$GRAFT_REPO_ROOT/ablib/lib_acc.so
    run v2-allfast . $c "$it" FITOCT_LIB_PATH=$GRAFT_REPO_ROOT/ablib/lib_v2.so
  done
done
