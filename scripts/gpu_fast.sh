#!/bin/bash
# GPU-box iteration on the fast kernel: full -m gpu suite, config-1 / config-2 bench lines,
# rocprofv3 kernel stats of the config-1 bench, phase stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/bench.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench.log | cut -c1-600
timeout -k 10 300 python bench.py --config 2 --steps 100 --warmup 10 --no-cpu --no-pmc --no-variant > gpurun_out/bench_cfg2.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg2.log | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --no-cpu --no-pmc --no-variant > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
find gpurun_out/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -6
timeout -k 10 200 python scripts/diag_phases.py > gpurun_out/diag_phases.json 2> gpurun_out/diag_phases.err || exit 1
echo diag ok
