#!/bin/bash
# HBM traffic of the sampler kernel from rocprofv3 PMC counters, one counter
# group per pass (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950),
# kernel-trace only.  Usage: pmc_traffic.sh [config] (BASELINE config, default 3).
# Writes gpurun_out/pmc_traffic_c<config>/* ; the summary JSON (workload named as the
# bench line names it) is copied to profiles/r<NN>_pmc_traffic_config<K>.json by hand,
# where bench.py finds it by workload.
set -e
CFG=${1:-3}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_traffic_c$CFG
mkdir -p $OUT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu --no-hard > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/pmc_summarize.py $OUT > $OUT/summary.json
cat $OUT/summary.json
