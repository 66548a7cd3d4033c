#!/bin/bash
# Round 4: A/B of the current library against abtest/lib_*.so variants (FITOCT_LIB_PATH) and the
# round-3 tree (abtest/r3): config 3 full length interleaved twice, then configs 2 and 5
# (2 steps each, interleaved twice).  Outputs gpurun_out/r4ablibs/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4ablibs
mkdir -p $OUT
run() {   # name dir env args
  (cd $2 && env $3 timeout -k 10 300 python3 bench.py $4 --no-cpu --no-hard 2>>$OUT/ab.err) | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$1 $4', d['value'], d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])" >> $OUT/ab.txt
}
variants() {
  run r4 $GRAFT_REPO_ROOT "FITOCT_NOP=1" "$1" || return 1
  for l in $GRAFT_REPO_ROOT/abtest/lib_*.so; do
    n=$(basename $l .so); run ${n#lib_} $GRAFT_REPO_ROOT "FITOCT_LIB_PATH=$l" "$1" || return 1
  done
  [ -d $GRAFT_REPO_ROOT/abtest/r3 ] && { run r3 $GRAFT_REPO_ROOT/abtest/r3 "FITOCT_NOP=1" "$1" || return 1; }
  return 0
}
for rep in 1 2; do variants "--steps 1 --warmup 0" || exit 1; done
for rep in 1 2; do for c in 2 5; do variants "--config $c --steps 2 --warmup 1" || exit 1; done; done
cat $OUT/ab.txt
