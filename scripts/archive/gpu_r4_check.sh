#!/bin/bash
# Round 4: quick check after a change to the two-ended path's waits: bitwise spec tests, batch
# tests, config 2's bench line.  Outputs gpurun_out/r4chk/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r4chk
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_batch.py tests/test_gpu_multidevice.py -q --timeout 300 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python3 bench.py --config 2 --steps 2 --warmup 1 --no-cpu > $OUT/config2.json 2> $OUT/config2.err || { tail -5 $OUT/config2.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/config2.json'));print('config 2', d['value'], d['roofline']['frac'], d['rhat_max'])"
