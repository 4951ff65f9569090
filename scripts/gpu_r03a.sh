#!/bin/bash
# Round-3 iteration: contact-form tests (incl. the 8f-2 extensions), the full GPU suite, config-1
# bench and a kernel-stats profile (follow-up launch cost).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_contact_ext.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_ext.log 2>&1
rc=$?; tail -n 15 gpurun_out/pytest_ext.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 5 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/bench.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench.log | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --no-cpu --no-pmc > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || exit 1
cut -d, -f1-4 "$GRAFT_REPO_ROOT/gpurun_out/prof/run_kernel_stats.csv" | head -8
