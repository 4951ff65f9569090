#!/bin/bash
# Round-3: chunked RowStore dots (n > 32 active set) -- full GPU suite, dummy drivers (stress p99),
# phase diagnostics (n = 39 repair / active loop), config-1 n = 39 line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 4 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 200 ./qppvm_amd/qppvm_dummy_driver --ticks 10000 > gpurun_out/dummy_qppvm.log 2>&1 || exit 1
timeout -k 10 200 ./qppvm_amd/qppvm_dummy_driver --ticks 10000 --stress > gpurun_out/dummy_qppvm_stress.log 2>&1 || exit 1
timeout -k 10 200 ./qppvm_amd/qppvm_dummy_driver --plugin forceacc --ticks 10000 > gpurun_out/dummy_forceacc.log 2>&1 || exit 1
tail -n 3 gpurun_out/dummy_*.log
timeout -k 10 300 python scripts/diag_phases.py > gpurun_out/diag_phases.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --n 39 --no-cpu --no-pmc --no-variant > gpurun_out/bench_n39.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_n39.log | cut -c1-400
exit $rc
