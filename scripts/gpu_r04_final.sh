#!/bin/bash
# round-4 evidence: default bench (config 1, PMC traffic, CPU baselines), rocprofv3 kernel stats of
# config 1 and config 4, smoke
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_final.log 2>&1 || { tail -n 5 gpurun_out/bench_final.log; exit 1; }
tail -n 1 gpurun_out/bench_final.log | cut -c1-600
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_c1" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 10 --no-cpu --no-pmc > "$GRAFT_REPO_ROOT/gpurun_out/prof_c1.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_c4" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --config 4 --steps 5 --warmup 1 --no-cpu --no-pmc > "$GRAFT_REPO_ROOT/gpurun_out/prof_c4.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
for d in prof_c1 prof_c4; do f=$(find gpurun_out/$d -name "*kernel_stats.csv" | head -1); echo "== $d"; cut -c1-160 "$f" | head -8; done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail -n 5 gpurun_out/smoke_final.log; exit 1; }
tail -n 2 gpurun_out/smoke_final.log
