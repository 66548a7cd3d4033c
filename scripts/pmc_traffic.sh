#!/bin/bash
# HBM traffic of the sampler kernel from rocprofv3 PMC counters, one counter
# group per pass (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950),
# kernel-trace only.  Writes gpurun_out/pmc_traffic/* ; the summary JSON is
# copied to profiles/ by hand.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_traffic
mkdir -p $OUT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/pmc_summarize.py $OUT > $OUT/summary.json
cat $OUT/summary.json
