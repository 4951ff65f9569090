#!/bin/bash
# GPU-box check: parity tests, smoke, bench, rocprof summary. Every GPU step has its own
# time limit; a crash / fault / timeout (exit >= 2 from pytest, or any non-zero from the
# others) ends the script there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-all}
run() { # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" ; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  return $rc
}
run pytest_gpu 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread ; rc=$?
if [ $rc -ge 2 ]; then echo "pytest crashed/timed out ($rc): stopping"; exit $rc; fi
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench 400 python bench.py --steps 200 --warmup 20 || exit 1
if [ "$STEPS" = "all" ]; then
  run bench_cfg2 300 python bench.py --config 2 --steps 100 --warmup 10 --no-cpu --no-variant || exit 1
  run bench_contact_cfg2 300 python bench.py --form contact --config 2 --steps 100 --warmup 10 --no-cpu || exit 1
  run bench_w1m 300 python bench.py --weight M --steps 100 --warmup 10 --no-cpu --no-variant || exit 1
  run bench_w1m_cfg2 300 python bench.py --weight M --config 2 --steps 50 --warmup 5 --no-cpu --no-variant || exit 1
  run bench_n39 300 python bench.py --n 39 --steps 100 --warmup 10 --no-cpu --no-variant || exit 1
  run bench_cfg4 300 python bench.py --config 4 --steps 20 --warmup 2 --cpu-seconds 10 --no-variant || exit 1
  run bench_cfg4_survey 300 python bench.py --config 4 --mpc-inputs survey --steps 5 --warmup 1 --no-cpu --no-pmc --no-variant || exit 1
  cd /tmp && run_dir="$GRAFT_REPO_ROOT/gpurun_out/prof"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$run_dir" -o run --output-format csv -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --no-cpu --no-pmc > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
  echo "prof rc=$?"; tail -n 2 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
fi
if [ "$STEPS" = "all" ] || [ "$STEPS" = "plugin" ]; then
  cd "$GRAFT_REPO_ROOT"
  run dummy_driver 300 ./qppvm_amd/qppvm_dummy_driver --ticks 10000 || exit 1
  run dummy_driver_stress 300 ./qppvm_amd/qppvm_dummy_driver --ticks 10000 --stress || exit 1
  run dummy_driver_forceacc 300 ./qppvm_amd/qppvm_dummy_driver --plugin forceacc --ticks 10000 || exit 1
fi
