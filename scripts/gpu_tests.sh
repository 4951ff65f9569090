#!/bin/bash
# GPU tests given as arguments (default: the whole gpu suite), one pytest process, own time limit.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 ${TLIM:-600} python -u -m pytest ${@:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_sel.log | tail -40
exit $rc
