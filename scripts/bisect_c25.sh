#!/bin/bash
# Bisect configs 2 and 5 across commit snapshots copied into abtest/wt_<hash>/ (each with its
# own bench.py, package and built libfitoct.so); "head" is the working tree.  Interleaved twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
out=gpurun_out/bisect_c25.txt; : > $out
for rep in 1 2; do
  for c in ${BISECT_CONFIGS:-2 5}; do
    for d in abtest/wt_* .; do
      [ -f $d/bench.py ] || continue
      r=$(cd $d && timeout -k 10 120 python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu 2>/dev/null) || { echo "$d config $c FAILED" >> $out; exit 1; }
      echo "$d config $c $(echo "$r" | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['roofline']['kernel_ms'])")" | tee -a $out
    done
  done
done
