#!/bin/bash
# Short GPU iteration: parity tests, config-1/2 bench, dummy-driver kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/bench.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench.log | cut -c1-400
timeout -k 10 300 python bench.py --config 2 --steps 100 --warmup 10 --no-cpu > gpurun_out/bench_cfg2.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_cfg2.log | cut -c1-400
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_dd" -o run --output-format csv -- \
    "$GRAFT_REPO_ROOT/qppvm_amd/qppvm_dummy_driver" --ticks 300 > "$GRAFT_REPO_ROOT/gpurun_out/prof_dd.log" 2>&1 || exit 1
tail -n 1 "$GRAFT_REPO_ROOT/gpurun_out/prof_dd.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- \
    python "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || exit 1
echo prof ok
