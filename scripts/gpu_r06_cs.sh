#!/bin/bash
# Round-6 constraint-space dual loop: parity subset on the product, lap counters of the stamp build
# (scripts/diag_gi.py), A/B of the product against abv/*.so on configs 1, 2 and 4. Each GPU step has its own
# limit; the first failure ends the script.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_gpu_parity.py tests/test_gpu_kkt.py tests/test_gpu_warmstart.py tests/test_gpu_rollout.py tests/test_gpu_followup.py tests/test_gpu_handback.py"}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sub.log 2>&1
  rc=$?; tail -n 3 gpurun_out/pytest_sub.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -f qppvm_amd/libwbq_diag.so ] && [ -z "${NODIAG:-}" ]; then
  timeout -k 10 200 python -u scripts/diag_gi.py > gpurun_out/diag_gi.log 2>&1 || { echo "diag rc=$?"; exit 1; }
  echo "diag ok"
fi
C4=1 bash scripts/gpu_ab.sh || exit 1
