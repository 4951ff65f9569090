#!/bin/bash
# GPU-box: config-0 plugin checks -- the plugin / parity tests, both dummy drivers (nominal and
# stress plants), and the per-tick phase diagnostics of the stress plant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_plugin.py tests/test_gpu_parity.py tests/test_gpu_w1m.py tests/test_gpu_kkt.py \
    -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_plugin.log 2>&1
rc=$?; tail -n 5 gpurun_out/pytest_plugin.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 200 ./qppvm_amd/qppvm_dummy_driver --ticks 10000 > gpurun_out/dummy_qppvm.log 2>&1 || exit 1
timeout -k 10 200 ./qppvm_amd/qppvm_dummy_driver --ticks 10000 --stress > gpurun_out/dummy_qppvm_stress.log 2>&1 || exit 1
timeout -k 10 200 ./qppvm_amd/qppvm_dummy_driver --plugin forceacc --ticks 10000 > gpurun_out/dummy_forceacc.log 2>&1 || exit 1
cat gpurun_out/dummy_*.log
DIAG_STRESS=1 DIAG_TICKS=30 timeout -k 10 200 python scripts/diag_plugin_tick.py gpurun_out/diag_tick.json > gpurun_out/diag_tick_stress.log 2>&1 || exit 1
tail -n 4 gpurun_out/diag_tick_stress.log
exit $rc
