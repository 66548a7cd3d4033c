#!/bin/bash
# Round 5, first check of the tree: the GPU tests this round changed or added, then a
# same-box A/B of config 3 at full length (HEAD against the round-4 final tree b170213,
# whose headline kernel spilled 2 VGPRs, and ddd35ce^ = 50ec006, the last round-4 tree
# without that spill), two interleaved runs each.  Outputs gpurun_out/r5check/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5check
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_spec.py tests/test_gpu_funnel.py::test_config5_file_rhat_distribution_matches_oracle \
  "tests/test_gpu_sampler.py::test_headline_shape_hard_geometry_rhat_below_1_01" \
  > $OUT/pytest.log 2>&1
rc=$?
tail -15 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for t in . ablib/wt_b170213 ablib/wt_50ec006; do
    (cd $t && timeout -k 10 200 python3 bench.py --config 3 --steps 1 --warmup 0 --no-cpu --no-hard \
       2>>$GRAFT_REPO_ROOT/$OUT/ab_stderr.log) > $OUT/ab.json || exit 1
    python3 -c "import json;d=json.load(open('$OUT/ab.json'));print('$t run $r', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])" | tee -a $OUT/ab.txt
  done
done
