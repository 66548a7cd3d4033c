#!/bin/bash
# Round 4: full-length A/B of config 3, split tile with speculation at every leaf
# (FITOCT_SPLIT=1 FITOCT_SPEC_LIVE=4) against the default 8-bin layout, interleaved twice;
# then the hard-geometry R-hat of the default path over step seeds.  Outputs gpurun_out/r4ab/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4ab
mkdir -p $OUT
for rep in 1 2; do
  for v in split_live4 nosplit; do
    envs="FITOCT_NOP=1"; [ $v = split_live4 ] && envs="FITOCT_SPLIT=1 FITOCT_SPEC_LIVE=4"
    env $envs timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu --no-hard 2>>$OUT/ab.err | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v full', d['value'], d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'rhat', d['rhat_max'], d['rank_rhat_max'], 'stuck', d['stuck_chains'])" >> $OUT/ab.txt || exit 1
  done
done
cat $OUT/ab.txt
timeout -k 10 600 python3 -u scripts/hard_seeds.py 1001 1019 1002 1003 1004 > $OUT/hard_seeds.jsonl 2> $OUT/hard_seeds.err || { tail -20 $OUT/hard_seeds.err; exit 1; }
cat $OUT/hard_seeds.jsonl
