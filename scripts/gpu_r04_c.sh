#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_cfg4.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg4.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg4" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config 4 --steps 5 --warmup 1 --no-cpu --no-pmc > "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg4.log" 2>&1 || exit 1
find "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg4" -name '*kernel_stats.csv' -exec cat {} \;
