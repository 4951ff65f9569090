#!/bin/bash
# Round-2 GPU check: the -m gpu suite (verbose, per-test timeout), then the config-0 dummy
# drivers and a kernel trace of the QPPVMPlugin tick loop. Every GPU step has its own limit;
# the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 30 "gpurun_out/$name.log"
  return $rc
}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"}; rc=$?
  [ $rc -ne 0 ] && { echo "pytest failed ($rc): stopping"; exit $rc; }
fi
if [ "${PLUGIN:-1}" = "1" ]; then
  run dummy_driver 300 ./qppvm_amd/qppvm_dummy_driver --ticks 10000 || exit 1
  run dummy_driver_forceacc 300 ./qppvm_amd/qppvm_dummy_driver --plugin forceacc --ticks 10000 || exit 1
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_plugin" -o run --output-format csv -- \
      "$R/qppvm_amd/qppvm_dummy_driver" --ticks 2000 > "$R/gpurun_out/prof_plugin.log" 2>&1
  echo "prof_plugin rc=$?"; tail -n 3 "$R/gpurun_out/prof_plugin.log"
  cd "$R"
fi
