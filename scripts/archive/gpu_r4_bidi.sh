#!/bin/bash
# Round 4: two-ended trajectories (P.bidi) -- the bitwise tests first, then config 2 with and
# without (FITOCT_NO_BIDI=1), 4 steps each, interleaved twice.  Outputs gpurun_out/r4bidi/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4bidi
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_spec.py -x -v --timeout 200 --timeout-method thread -m gpu -k "two_ended or speculative_leaves_preserve or batch_of_one" > $OUT/pytest.log 2>&1; rc=$?
tail -15 $OUT/pytest.log
if [ $rc -ne 0 ]; then
  [ $rc -eq 1 ] && timeout -k 10 120 python -u scripts/bidi_diag.py > $OUT/diag.log 2>&1; cat $OUT/diag.log
  exit $rc
fi
run() {   # name env args
  env $2 timeout -k 10 300 python3 bench.py $3 --no-cpu --no-hard 2>>$OUT/ab.err | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$1 $3', d['value'], d['roofline']['kernel_ms'], 'TF', d['roofline']['achieved'], 'frac', d['roofline']['frac'], 'R-hat', d.get('rhat_max'))" >> $OUT/ab.txt
}
for rep in 1 2; do
  run bidi "FITOCT_NOP=1" "--config 2 --steps 4 --warmup 1" || exit 1
  run nobidi "FITOCT_NO_BIDI=1" "--config 2 --steps 4 --warmup 1" || exit 1
done
cat $OUT/ab.txt
