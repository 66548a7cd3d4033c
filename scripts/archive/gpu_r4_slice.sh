#!/bin/bash
# (Historical: the NUTS-wave slice was measured with this script and removed, profiles/r04_ab_nuts_slice.txt;
# on later trees FITOCT_NUTS_SLICE does nothing.)
# Round 4: NUTS-wave slice (FITOCT_NUTS_SLICE = 2 / 4: the last 2 / 4 of the 8 bins per
# gradient lane swept by each chain's own NUTS wave from L2) against the default, config 3:
# short runs interleaved twice, then full length; a parity test of the slice path.
# Outputs gpurun_out/r4slice/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4slice
mkdir -p $OUT
run() {   # name env args
  env $2 timeout -k 10 300 python3 bench.py $3 --no-cpu --no-hard 2>>$OUT/ab.err | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$1 $3', d['value'], d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'stuck', d['stuck_chains'], 'rhat', d['rhat_max'])" >> $OUT/ab.txt
}
for rep in 1 2; do
  run base "FITOCT_NOP=1" "--steps 2 --warmup 1 --iters 200,200" || exit 1
  run slice2 "FITOCT_NUTS_SLICE=2" "--steps 2 --warmup 1 --iters 200,200" || exit 1
  run slice4 "FITOCT_NUTS_SLICE=4" "--steps 2 --warmup 1 --iters 200,200" || exit 1
done
cat $OUT/ab.txt
for v in base slice2; do
  e="FITOCT_NOP=1"; [ $v = slice2 ] && e="FITOCT_NUTS_SLICE=2"
  run $v "$e" "--steps 1 --warmup 0" || exit 1
done
cat $OUT/ab.txt
FITOCT_NUTS_SLICE=2 timeout -k 10 300 python -u -m pytest "tests/test_gpu_sampler.py::test_headline_shape_converges_and_matches_oracle[1000]" tests/test_gpu_funnel.py::test_headline_funnel_trapping_matches_oracle -x -q --timeout 250 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1; tail -5 $OUT/pytest.log
