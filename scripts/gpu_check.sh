#!/bin/bash
# GPU-box check, in two parts (one gpurun call each): STEPS=a  parity tests, smoke, the bench lines of
# configs 1 / 2 / 4 and their rocprofv3 kernel statistics; STEPS=b  the other bench lines (W1 = M, n = 39,
# contact config 2), the config-1 phase stamps, the plugin shells in dummy mode, the stress-plant tick split.
# Every GPU step has its own time limit; a crash / fault / timeout ends the script there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-a}
run() { # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" ; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-300
  return $rc
}
if [ "$STEPS" = "a" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 180 --timeout-method thread ; rc=$?
  if [ $rc -ne 0 ]; then echo "pytest failed ($rc): stopping"; exit $rc; fi
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
  run bench 400 python bench.py --steps 200 --warmup 20 || exit 1
  run bench_cfg2 300 python bench.py --config 2 --steps 100 --warmup 10 --no-cpu --no-variant || exit 1
  run bench_cfg4 300 python bench.py --config 4 --steps 20 --warmup 2 --cpu-seconds 10 --no-variant || exit 1
  cd /tmp
  for cfg in 1 2 4; do # kernel statistics of the bench configurations (the bench lines' event times beside them)
    st=200; [ $cfg = 4 ] && st=10
    # (one launch shape per summary: no contact-form variant, and config 4 without the one-step launches of the
    # repair-share pass)
    ex="--no-variant"; [ $cfg = 4 ] && ex="--no-variant --no-repair-share"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_cfg$cfg" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" --config $cfg --steps $st --warmup 5 --no-cpu --no-pmc $ex > "$ROOT/gpurun_out/prof_cfg$cfg.log" 2>&1
    rc=$?; echo "prof cfg$cfg rc=$rc"
    [ $rc -ne 0 ] && exit 1
  done
  cd "$ROOT"
fi
if [ "$STEPS" = "b" ]; then
  run bench_w1m_cfg2 300 python bench.py --weight M --config 2 --steps 50 --warmup 5 --no-cpu --no-variant || exit 1
  run bench_w1m 300 python bench.py --weight M --steps 100 --warmup 10 --no-cpu --no-variant || exit 1
  run bench_n39 300 python bench.py --n 39 --steps 100 --warmup 10 --no-cpu --no-variant || exit 1
  run bench_contact_cfg2 300 python bench.py --form contact --config 2 --steps 100 --warmup 10 --no-cpu || exit 1
  run diag_phases 300 python -u scripts/diag_phases.py || exit 1
  run dummy_driver 300 ./qppvm_amd/qppvm_dummy_driver --ticks 10000 || exit 1
  run dummy_driver_stress 300 ./qppvm_amd/qppvm_dummy_driver --ticks 10000 --stress || exit 1
  run dummy_driver_forceacc 300 ./qppvm_amd/qppvm_dummy_driver --plugin forceacc --ticks 10000 || exit 1
  DIAG_STRESS=1 DIAG_TICKS=400 run diag_tick_stress 300 python -u scripts/diag_plugin_tick.py gpurun_out/diag_tick_stress.json || exit 1
fi
