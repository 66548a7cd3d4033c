#!/bin/bash
# Round 6: finish_grad without the SUMS round trip in row mode, Chain<..., MODE> (basis mode
# a compile-time constant of the sampler) -- suites on the new library, then A/B vs HEAD.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/ab_fg}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  ${TESTS:-tests/test_gpu_logp.py tests/test_gpu_pair.py tests/test_gpu_batch.py tests/test_gpu_spec.py tests/test_gpu_migration.py} > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
OUT=$OUT LIBS="${LIBS:-head:prof6/lib_rowsbase.so new}" CONFIGS="${CONFIGS:-2 3 5}" REPS="1 2" bash scripts/gpu_ab.sh
