#!/bin/bash
# PMC passes (one counter group per pass), kernel-trace only; writes gpurun_out/pmc/*
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
i=0
for grp in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAVES" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" ; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 scripts/prof_small.py > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
done
for f in $(find gpurun_out/pmc -name "*counter_collection.csv"); do echo $f; python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float)
for r in rows:
    if 'nuts_kernel' in r.get('Kernel_Name',''):
        agg[r['Counter_Name']] += float(r['Counter_Value'])
for k, v in sorted(agg.items()): print(f"  {k} = {v:.4g}")
PY
done
