#!/bin/bash
# Round 5: same-box A/B of migrating-sampler register variants (ablib/lib_A: fexp three-VGPR
# FMAs; lib_B: the speculated leaf kept in registers; lib_C: both) against HEAD, config 3 at
# full length (interleaved twice) and config 4 once.  gpurun_out/r5migvar/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5migvar
mkdir -p $OUT
run() {   # label, config, env...
  local l=$1; local c=$2; shift; shift
  env "$@" timeout -k 10 200 python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu --no-hard \
    2>>$OUT/stderr.log > $OUT/ab.json || exit 1
  python3 -c "import json;d=json.load(open('$OUT/ab.json'));print('$l config $c', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" | tee -a $OUT/ab.txt
}
for r in 1 2; do
  run head 3 FITOCT_X=0
  for v in A B C; do run $v 3 FITOCT_LIB_PATH=$PWD/ablib/lib_$v.so; done
done
run head 4 FITOCT_X=0
for v in A B C; do run $v 4 FITOCT_LIB_PATH=$PWD/ablib/lib_$v.so; done
