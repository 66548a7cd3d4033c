#!/bin/bash
# Round 4: Estrin (lat_all: every <= 2-bin sweep; lat_nospec: only kernels without speculation) forms in the <= 2-bins-per-lane sweeps (FITOCT_LAT_SWEEP, default on) against
# abtest/lib_nolat.so (Horner), configs 2 and 5: 4 steps (4 seeds) each, interleaved twice; the
# per-gradient rate ('TF') compares across the two arithmetic variants.  Then the lp / gradient
# and sampler parity tests on the new forms.  Outputs gpurun_out/r4lat/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4lat
mkdir -p $OUT
run() {   # name env args
  env $2 timeout -k 10 300 python3 bench.py $3 --no-cpu --no-hard 2>>$OUT/ab.err | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$1 $3', d['value'], d['roofline']['kernel_ms'], 'TF', d['roofline']['achieved'], 'frac', d['roofline']['frac'])" >> $OUT/ab.txt
}
for rep in 1 2; do
  for c in 2 5; do
    run lat_nospec "FITOCT_NOP=1" "--config $c --steps 4 --warmup 1" || exit 1
    run lat_all "FITOCT_LIB_PATH=$GRAFT_REPO_ROOT/abtest/lib_latall.so" "--config $c --steps 4 --warmup 1" || exit 1
    run nolat "FITOCT_LIB_PATH=$GRAFT_REPO_ROOT/abtest/lib_nolat.so" "--config $c --steps 4 --warmup 1" || exit 1
  done
done
run main "FITOCT_NOP=1" "--steps 2 --warmup 1" || exit 1
run nolat "FITOCT_LIB_PATH=$GRAFT_REPO_ROOT/abtest/lib_nolat.so" "--steps 2 --warmup 1" || exit 1
cat $OUT/ab.txt
[ -n "$NO_TESTS" ] && exit 0
timeout -k 10 600 python -u -m pytest tests/test_gpu_logp.py tests/test_gpu_sampler.py tests/test_gpu_batch.py tests/test_gpu_spec.py -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1; tail -3 $OUT/pytest.log
