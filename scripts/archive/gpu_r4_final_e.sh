#!/bin/bash
# Round-4 final tree (two-ended trajectories with lookahead 3 and extended rings): the whole GPU
# suite, smoke(), the default bench line, its rocprofv3 kernel stats, and the secondary lines of
# configs 2, 4, 5.  Outputs gpurun_out/r4fe/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4fe
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('config 3', d['value'], d['roofline']['frac'], d['hard_geometry']['rhat_max'], d['hard_geometry']['rank_rhat_max'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-hard > $OUT/trace.out 2>&1 || { tail -5 $OUT/trace.out; exit 1; }
for c in 2 4 5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu > $OUT/config$c.json 2> $OUT/config$c.err || { tail -5 $OUT/config$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/config$c.json'));print('config $c', d['value'], d['roofline']['frac'])"
done
