#!/bin/bash
# Round-6 GPU step: the parity subset that covers the fast path, then same-box A/B of the product against
# abv/*.so (configs 1, 2, 4) and a rocprofv3 kernel-trace summary of config 1. Each GPU step has its own limit.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_gpu_parity.py tests/test_gpu_kkt.py tests/test_gpu_warmstart.py tests/test_gpu_rollout.py tests/test_gpu_followup.py"}
if [ -n "$TESTS" ] && [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sub.log 2>&1
  rc=$?; tail -n 5 gpurun_out/pytest_sub.log; [ $rc -ne 0 ] && exit $rc
fi
C4=${C4:-1} bash scripts/gpu_ab.sh || exit 1
if [ -n "${SMALLB:-}" ]; then # the per-wave chain: one wave per SIMD or less (B = 256, 1024)
  for lib in qppvm_amd/libwbq.so abv/*.so; do
    for B in 256 1024; do
      timeout -k 10 120 python scripts/ab_bench.py "$lib" --batch $B --steps 200 --warmup 20 --no-cpu --no-pmc --no-variant > gpurun_out/ab_$(basename $lib .so)_b$B.log 2>&1 || exit 1
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['roofline']['kernel_avg_us'],2), 'us')" gpurun_out/ab_$(basename $lib .so)_b$B.log
    done
  done
fi
if [ -n "${PROF:-}" ]; then
  cd /tmp
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg1" -o run --output-format csv -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --no-cpu --no-pmc --no-variant > "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg1.log" 2>&1
  echo "prof rc=$?"
fi
