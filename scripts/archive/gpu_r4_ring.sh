#!/bin/bash
# Round 4: two-ended trajectories with rings extended into the producers' tree-level areas --
# the bitwise tests, then config 2 against rings capped at the previous 52 records.
# Outputs gpurun_out/r4ring/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4ring
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_spec.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
run() {   # name env args
  env $2 timeout -k 10 300 python3 bench.py $3 --no-cpu --no-hard 2>>$OUT/ab.err | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$1 $3', d['value'], d['roofline']['kernel_ms'], 'TF', d['roofline']['achieved'], 'R-hat', d.get('rhat_max'))" >> $OUT/ab.txt
}
for rep in 1 2; do
  run ring_full "FITOCT_NOP=1" "--config 2 --steps 4 --warmup 1" || exit 1
  run ring52 "FITOCT_BIDI_RB=52" "--config 2 --steps 4 --warmup 1" || exit 1
done
cat $OUT/ab.txt
