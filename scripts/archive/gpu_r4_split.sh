#!/bin/bash
# (Historical: the split tile was measured with this script at commit 1a05d88 and then removed,
# profiles/r04_ab_split.txt; on a later tree FITOCT_SPLIT does nothing.)
# Round 4: split tile (kernel_params.h gsplit: 16 bins per lane over half the gradient waves
# per chain at the headline shape).  Parity and bitwise tests on the new layout, then an
# interleaved A/B of config 3 without FITOCT_SPLIT=1 (the 8-bin layout, same library):
# short runs (200 + 200) and one full-length step each.  Outputs gpurun_out/r4split/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4split
mkdir -p $OUT
FITOCT_SPLIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_spec.py tests/test_gpu_migration.py tests/test_gpu_logp.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
for rep in 1 2; do
  for v in split nosplit split_live2 split_live4; do
    case $v in
      split) envs="FITOCT_SPLIT=1" ;;
      nosplit) envs="FITOCT_NOP=1" ;;
      split_live2) envs="FITOCT_SPLIT=1 FITOCT_SPEC_LIVE=2" ;;
      split_live4) envs="FITOCT_SPLIT=1 FITOCT_SPEC_LIVE=4" ;;
    esac
    env $envs timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-hard --iters 200,200 2>>$OUT/ab.err | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v short', d['value'], d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])" >> $OUT/ab.txt || exit 1
  done
done
for v in split nosplit; do
  envs="FITOCT_NOP=1"; [ $v = split ] && envs="FITOCT_SPLIT=1"
  env $envs timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu --no-hard 2>>$OUT/ab.err | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v full', d['value'], d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'rhat', d['rhat_max'], d['rank_rhat_max'], 'stuck', d['stuck_chains'])" >> $OUT/ab.txt || exit 1
done
cat $OUT/ab.txt
