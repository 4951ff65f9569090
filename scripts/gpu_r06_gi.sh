#!/bin/bash
# Round-6 dual_gi.h (contact form, W1 = M) with wave-ordered LDS: the tests of those paths, then same-box A/B of the
# product against abv/*.so on the contact form (configs 1 and 2) and W1 = M (configs 1 and 2). Each GPU step has
# its own limit; the first failure ends the script.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_gpu_contact.py tests/test_gpu_contact_ext.py tests/test_gpu_w1m.py tests/test_gpu_kkt.py"}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 700 python -u -m pytest $TESTS -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gi.log 2>&1
  rc=$?; tail -n 3 gpurun_out/pytest_gi.log; [ $rc -ne 0 ] && exit $rc
fi
for lib in qppvm_amd/libwbq.so abv/*.so; do
  nm=$(basename "$lib" .so)
  timeout -k 10 200 python scripts/ab_bench.py "$lib" --form contact --steps 100 --warmup 10 --no-cpu --no-pmc > gpurun_out/gi_${nm}_k1.log 2>&1 || exit 1
  timeout -k 10 200 python scripts/ab_bench.py "$lib" --form contact --config 2 --steps 40 --warmup 5 --no-cpu --no-pmc > gpurun_out/gi_${nm}_k2.log 2>&1 || exit 1
  timeout -k 10 200 python scripts/ab_bench.py "$lib" --weight M --steps 100 --warmup 10 --no-cpu --no-pmc --no-variant > gpurun_out/gi_${nm}_m1.log 2>&1 || exit 1
  timeout -k 10 200 python scripts/ab_bench.py "$lib" --weight M --config 2 --steps 30 --warmup 5 --no-cpu --no-pmc --no-variant > gpurun_out/gi_${nm}_m2.log 2>&1 || exit 1
  python - "$nm" <<'PY'
import json, sys
nm = sys.argv[1]
for c in ("k1", "k2", "m1", "m2"):
    d = json.loads(open(f"gpurun_out/gi_{nm}_{c}.log").read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    print(f"{nm:12s} {c} {d['value']/1e6:8.2f} M/s  step {d['ms_per_step']*1e3:8.1f} us  kernel {r.get('kernel_avg_us', 0):8.1f} us  "
          f"steps mean {d.get('mean_active_set_steps')} max {d.get('max_active_set_steps')}")
PY
done
