#!/bin/bash
# Round 5: two-ended trajectories in the migrating launch's tail.  GPU tests of the paths
# this touches, then config 3 at full length with and without it (FITOCT_NO_TAIL_BIDI=1),
# interleaved, and two tail thresholds.  Outputs gpurun_out/r5tail/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5tail
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_migration.py tests/test_gpu_spec.py tests/test_gpu_smoke.py tests/test_gpu_logp.py \
  > $OUT/pytest.log 2>&1
rc=$?
tail -30 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
run() {   # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --config 3 --steps 1 --warmup 0 --no-cpu --no-hard \
    2>>$OUT/ab_stderr.log > $OUT/ab.json || exit 1
  python3 -c "import json;d=json.load(open('$OUT/ab.json'));print('$l', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['rhat_max'])" | tee -a $OUT/ab.txt
}
for r in 1 2; do
  run "tail-on" FITOCT_X=0
  run "tail-off" FITOCT_NO_TAIL_BIDI=1
  run "tail-on-sweepfast" FITOCT_LIB_PATH=$PWD/ablib/lib_sweepfast.so
done
run5() {   # label, config, env...
  local l=$1; local c=$2; shift; shift
  env "$@" timeout -k 10 200 python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu \
    2>>$OUT/ab_stderr.log > $OUT/ab.json || exit 1
  python3 -c "import json;d=json.load(open('$OUT/ab.json'));print('$l config $c', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" | tee -a $OUT/ab.txt
}
for r in 1 2; do
  for c in 2 5; do
    run5 "sweep-on" $c FITOCT_X=0
    run5 "sweep-fast" $c FITOCT_LIB_PATH=$PWD/ablib/lib_sweepfast.so
  done
done
