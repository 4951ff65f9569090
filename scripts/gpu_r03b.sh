#!/bin/bash
# Round-3 iteration: the 8f-1 / 8f-2 tests first, then the full GPU suite and a config-1 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_contact_ext.py tests/test_gpu_rbd.py -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_new.log | tail -30; [ $rc -ge 2 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 8 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu --no-pmc > gpurun_out/bench.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench.log | cut -c1-200
