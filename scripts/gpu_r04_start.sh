#!/bin/bash
# Round-4 start-of-round check: GPU suite, headline bench, config-4 bench with a kernel trace.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -n 3 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-pmc > gpurun_out/bench.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench.log
timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_cfg4.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg4.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg4" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config 4 --steps 3 --warmup 1 --no-cpu --no-pmc > "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg4.log" 2>&1 || exit 1
find "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg4" -name '*kernel_stats.csv' -exec cat {} \;
