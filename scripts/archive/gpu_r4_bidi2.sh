#!/bin/bash
# Round 4: two-ended trajectories with the leaf rings in LDS -- the bitwise tests, config 2 with
# and without (FITOCT_NO_BIDI=1) interleaved twice, config 2's PMC traffic.  Outputs gpurun_out/r4bidi2/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4bidi2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_spec.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
run() {   # name env args
  env $2 timeout -k 10 300 python3 bench.py $3 --no-cpu --no-hard 2>>$OUT/ab.err | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$1 $3', d['value'], d['roofline']['kernel_ms'], 'TF', d['roofline']['achieved'], 'frac', d['roofline']['frac'], 'R-hat', d.get('rhat_max'))" >> $OUT/ab.txt
}
for rep in 1 2; do
  run bidi_lds "FITOCT_NOP=1" "--config 2 --steps 4 --warmup 1" || exit 1
  run nobidi "FITOCT_NO_BIDI=1" "--config 2 --steps 4 --warmup 1" || exit 1
done
cat $OUT/ab.txt
timeout -k 10 400 bash scripts/pmc_traffic.sh 2 > $OUT/pmc_c2.out 2>&1 || { tail -5 $OUT/pmc_c2.out; exit 1; }
tail -4 $OUT/pmc_c2.out
