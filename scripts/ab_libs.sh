#!/bin/bash
# A/B: every ablib/lib_*.so on the BASELINE configs (AB_CONFIGS, default "3 4 2 5"), short
# runs, interleaved twice.  Configs 2 and 5 end with their slowest chain / tile, which
# moves with any change to the arithmetic (chaotic trajectories): they run 4 seeds per
# line.  'TF' (algorithmic FP64 TFLOP/s = gradients x flop / kernel time) is the per-
# gradient rate, comparable across variants whose trajectories differ.  ablib/env_<name>
# (KEY=VALUE lines) is added to lib_<name>'s environment.
cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for c in ${AB_CONFIGS:-3 4 2 5}; do
    for l in ${AB_DIR:-ablib}/lib_*.so; do
      it="200,200"; st=1
      [ $c = 5 ] && it="100,100"
      { [ $c = 2 ] || [ $c = 5 ]; } && st=4
      n=$(basename $l .so); n=${n#lib_}
      envs=""; [ -f ${AB_DIR:-ablib}/env_$n ] && envs=$(cat ${AB_DIR:-ablib}/env_$n)
      env $envs FITOCT_LIB_PATH=$PWD/$l timeout -k 10 200 python3 bench.py --config $c --steps $st --warmup 1 --no-cpu --no-hard --iters $it 2>>gpurun_out/ab_stderr.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$l config $c', d['value'], d['roofline']['kernel_ms'], 'TF', d['roofline']['achieved'])" || exit 1
    done
  done
done
