#!/bin/bash
# A/B at full length on the headline workload (config 3, 500 + 1000 iterations): effects
# on the launch's tail (load balance) do not show in the short runs of ab_libs.sh.
cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for l in ${AB_DIR:-ablib}/lib_*.so; do
    n=$(basename $l .so); n=${n#lib_}
    envs=""; [ -f ${AB_DIR:-ablib}/env_$n ] && envs=$(cat ${AB_DIR:-ablib}/env_$n)
    env $envs FITOCT_LIB_PATH=$PWD/$l timeout -k 10 200 python3 bench.py --config 3 --steps 1 --warmup 0 --no-cpu --no-hard 2>>gpurun_out/ab_stderr.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$l config 3 full', d['value'], d['roofline']['kernel_ms'], 'TF', d['roofline']['achieved'])" || exit 1
  done
done
