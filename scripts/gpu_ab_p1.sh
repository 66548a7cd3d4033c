#!/bin/bash
# Round 6: the chain's wave books the forward end of an unpaired row-mode tile -- suites, then
# config 2 unpaired / paired and config 5 (with its strong-scaling estimate) against HEAD.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/ab_p1}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_pair.py tests/test_gpu_spec.py tests/test_gpu_batch.py tests/test_gpu_migration.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
OUT=$OUT LIBS="hd:prof6/lib_hd.so:FITOCT_NO_PAIR=1 new::FITOCT_NO_PAIR=1 hdp:prof6/lib_hd.so newp" CONFIGS=2 REPS="1 2" bash scripts/gpu_ab.sh || exit 1
for r in 1 2; do for v in hd:prof6/lib_hd.so new:; do
  IFS=: read -r l lp <<< "$v"; [ -n "$lp" ] && lp=$PWD/$lp
  FITOCT_LIB_PATH=$lp timeout -k 10 300 python3 bench.py --config 5 --no-cpu > $OUT/c5.json 2>> $OUT/stderr.log || exit 1
  python3 -c "import json;d=json.load(open('$OUT/c5.json'));print('$l config 5', d['value'], [e['efficiency_est'] for e in d['strong_scaling_est']], [e['ms_per_step_est'] for e in d['strong_scaling_est']])"
done; done
