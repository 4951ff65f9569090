#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_contact_ext.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|sweep" gpurun_out/pytest_sel.log | tail -40
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 1 --no-cpu --no-pmc > gpurun_out/bench_cfg4.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg4.log
