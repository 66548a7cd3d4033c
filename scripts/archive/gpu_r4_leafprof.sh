#!/bin/bash
# Round 4: the latency-bound leaf path (configs 2 / 5) profiled: per-action / sub-action
# cycle stamps from the profiling build (abtest/lib_prof.so, FITOCT_PROFILE=1) at the config 2,
# config-5-like and config 3 shapes, and the per-gradient instruction mix from PMC counters
# (with and without the sweep).  Outputs gpurun_out/r4leaf/ and gpurun_out/pmc_leaf*/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4leaf
mkdir -p $OUT
FITOCT_LIB_PATH=$GRAFT_REPO_ROOT/abtest/lib_prof.so timeout -k 10 300 python3 scripts/stamps_actions.py > $OUT/stamps_actions.txt 2>&1 || { tail -20 $OUT/stamps_actions.txt; exit 1; }
FITOCT_LIB_PATH=$GRAFT_REPO_ROOT/abtest/lib_prof.so timeout -k 10 300 python3 scripts/stamps_speculative.py > $OUT/stamps_spec.txt 2>&1 || { tail -20 $OUT/stamps_spec.txt; exit 1; }
for pd in 0 1; do timeout -k 10 200 bash scripts/pmc_leaf.sh $pd > $OUT/pmc_leaf$pd.txt 2>&1 || { cat $OUT/pmc_leaf$pd.txt; exit 1; }; done
cat $OUT/pmc_leaf0.txt $OUT/pmc_leaf1.txt
grep -h "stamps\|kernel" $OUT/stamps_actions.txt | head -40
