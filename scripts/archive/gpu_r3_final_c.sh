#!/bin/bash
# Final tree check: the whole GPU suite and smoke() on the default library, bitwise draws of
# abtest/lib_*.so against lib_base, short-run rates of configs 2 and 5.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final_pytest.log 2>&1 || { tail -40 gpurun_out/final_pytest.log; exit 1; }
tail -2 gpurun_out/final_pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { cat gpurun_out/final_smoke.log; exit 1; }
grep -v amdgpu gpurun_out/final_smoke.log
timeout -k 10 400 python3 -u scripts/ab_bitwise.py > gpurun_out/fmav2_bitwise.txt 2>&1 || { cat gpurun_out/fmav2_bitwise.txt; exit 1; }
grep -v amdgpu gpurun_out/fmav2_bitwise.txt
AB_CONFIGS="2 5" timeout -k 10 500 bash scripts/ab_libs.sh > gpurun_out/fmav2_short.txt 2>&1 || { cat gpurun_out/fmav2_short.txt; exit 1; }
cat gpurun_out/fmav2_short.txt
