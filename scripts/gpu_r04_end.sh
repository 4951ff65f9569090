#!/bin/bash
# end of round 4: the whole GPU suite, smoke, the default bench line
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/pytest_end.log 2>&1; rc=$?
tail -n 2 gpurun_out/pytest_end.log; grep -n "^FAILED" gpurun_out/pytest_end.log | head -5
[ $rc -ge 2 ] && exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_end.log 2>&1 || { tail -n 5 gpurun_out/smoke_end.log; exit 1; }
tail -n 1 gpurun_out/smoke_end.log
timeout -k 10 600 python bench.py > gpurun_out/bench_end.log 2>&1 || { tail -n 5 gpurun_out/bench_end.log; exit 1; }
tail -n 1 gpurun_out/bench_end.log | cut -c1-400
