#!/bin/bash
# A/B (MODES: 0 = separate, 1 = inline, auto = by the last repair counts) of the level-0 repair inside the fast kernel (WBQ_INLREP=1, one launch per solve) against the
# separate qppvm_repair_kernel (WBQ_INLREP=0), same box: config 1, config 2, config 4 (plant and
# SURVEY inputs), then the repair / warm-start parity tests with the inline variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
summ() { python -c "
import json; d=json.loads(open('gpurun_out/$1.log').read().strip().splitlines()[-1])
print('$1', round(d['value']/1e6,3), 'M QP/s, step', round(d['ms_per_step']*1e3,2), 'us, kernel', round(d['roofline']['kernel_avg_us'],2), 'us', d['status_histogram'])"; }
run() { local v=$1; shift; if [ "$v" = auto ]; then env -u WBQ_INLREP "$@"; else WBQ_INLREP=$v "$@"; fi; }
for v in ${MODES:-0 auto}; do
  run $v timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu --no-pmc --no-variant > gpurun_out/inl${v}_c1.log 2>&1 || exit 1; summ inl${v}_c1
done
for v in ${MODES:-0 auto}; do
  run $v timeout -k 10 120 python bench.py --config 2 --steps 100 --warmup 10 --no-cpu --no-pmc --no-variant > gpurun_out/inl${v}_c2.log 2>&1 || exit 1; summ inl${v}_c2
  run $v timeout -k 10 120 python bench.py --config 4 --steps 10 --warmup 1 --no-cpu --no-pmc --no-variant > gpurun_out/inl${v}_c4.log 2>&1 || exit 1; summ inl${v}_c4
  run $v timeout -k 10 120 python bench.py --config 4 --mpc-inputs survey --steps 5 --warmup 1 --no-cpu --no-pmc --no-variant > gpurun_out/inl${v}_c4s.log 2>&1 || exit 1; summ inl${v}_c4s
done
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/inl_pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/inl_pytest.log; [ $rc -ne 0 ] && exit $rc
WBQ_INLREP=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rollout.py tests/test_gpu_warmstart.py tests/test_gpu_joint_limits.py tests/test_gpu_kkt.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/inl1_pytest.log 2>&1; rc=$?; tail -n 2 gpurun_out/inl1_pytest.log; exit $rc
