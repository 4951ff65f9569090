#!/bin/bash
# Round-6 u-space loop (n > 32) with wave-ordered LDS: the tests of those paths, then the config-0 stress plant and the
# n = 39 bench lines for the product and for abv/gs_head.so (swapped in place on the box's copy: the dummy driver
# loads the library next to it). Each GPU step has its own limit; the first failure ends the script.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_gpu_handback.py tests/test_gpu_elbow.py tests/test_plugin.py tests/test_gpu_parity.py"}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 700 python -u -m pytest $TESTS -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_n39.log 2>&1
  rc=$?; tail -n 3 gpurun_out/pytest_n39.log; [ $rc -ne 0 ] && exit $rc
fi
one() { # tag
  local t=$1
  timeout -k 10 300 ./qppvm_amd/qppvm_dummy_driver --ticks 10000 --stress > gpurun_out/n39_${t}_stress.log 2>&1 || exit 1
  tail -n 2 gpurun_out/n39_${t}_stress.log | cut -c1-300
  timeout -k 10 200 python bench.py --n 39 --steps 100 --warmup 10 --no-cpu --no-pmc --no-variant > gpurun_out/n39_${t}_c1.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --n 39 --config 2 --steps 50 --warmup 5 --no-cpu --no-pmc --no-variant > gpurun_out/n39_${t}_c2.log 2>&1 || exit 1
  python - "$t" <<'PY'
import json, sys
t = sys.argv[1]
for c in ("c1", "c2"):
    d = json.loads(open(f"gpurun_out/n39_{t}_{c}.log").read().strip().splitlines()[-1])
    print(f"{t:10s} n39 {c} {d['value']/1e6:8.2f} M/s  step {d['ms_per_step']*1e3:8.1f} us  steps mean {d.get('mean_active_set_steps')} max {d.get('max_active_set_steps')}")
PY
}
one product
if [ -f abv/gs_head.so ]; then
  cp abv/gs_head.so qppvm_amd/libwbq.so
  one gs_head
fi
