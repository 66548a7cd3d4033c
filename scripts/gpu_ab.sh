#!/bin/bash
# Same-box A/B of library variants on BASELINE configs at full length (round 5).
#   LIBS="new base:gpulib/lib_base.so off::FITOCT_X=1 ..."  (label[:path[:ENV=VAL]]; no path =
#   fitoct_amd/libfitoct.so)
#   CONFIGS="2 3"  REPS="1 2"  OUT=gpurun_out/ab  TESTS="tests/test_gpu_spec.py ..." (run first)
# Config 2 times 3 steps (its chains end with the slowest), config 3 one step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/ab}
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS \
    > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for r in ${REPS:-1 2}; do
  for c in ${CONFIGS:-2 3}; do
    for v in ${LIBS:-new}; do
      IFS=: read -r l lp ev <<< "$v"
      [ -n "$lp" ] && lp=$PWD/$lp
      st=1; [ $c = 2 ] && st=3
      env $ev FITOCT_LIB_PATH=$lp timeout -k 10 200 python3 bench.py --config $c --steps $st --warmup 1 --no-cpu --no-hard \
         2>>$OUT/stderr.log > $OUT/b.json || exit 1
      python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$l config $c', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" | tee -a $OUT/ab.txt
    done
  done
done
