#!/bin/bash
# The linear families' fused coefficient update: the whole GPU suite on the default library
# (fused), then short-run rates of configs 2, 5, 4 for abtest/lib_base.so (HEAD) and
# abtest/lib_fuse.so.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fuse_pytest.log 2>&1 || { tail -40 gpurun_out/fuse_pytest.log; exit 1; }
tail -2 gpurun_out/fuse_pytest.log
AB_CONFIGS="2 5 4" timeout -k 10 600 bash scripts/ab_libs.sh > gpurun_out/fuse_ab.txt 2>&1 || { cat gpurun_out/fuse_ab.txt; exit 1; }
cat gpurun_out/fuse_ab.txt
timeout -k 10 240 bash scripts/pmc_stall.sh 0 > gpurun_out/pmc_stall0.out 2>&1 || { tail -5 gpurun_out/pmc_stall0.out; exit 1; }
cat gpurun_out/pmc_stall0.out
