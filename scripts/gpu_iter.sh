set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu --no-pmc --no-variant > gpurun_out/b_c1.log 2>&1 || exit 1
tail -n 1 gpurun_out/b_c1.log | cut -c1-300
timeout -k 10 300 python bench.py --weight M --steps 100 --warmup 10 --no-cpu --no-pmc --no-variant > gpurun_out/b_w1m_c1.log 2>&1 || exit 1
tail -n 1 gpurun_out/b_w1m_c1.log | cut -c1-300
timeout -k 10 300 python bench.py --weight M --config 2 --steps 50 --warmup 5 --no-cpu --no-pmc --no-variant > gpurun_out/b_w1m_c2.log 2>&1 || exit 1
tail -n 1 gpurun_out/b_w1m_c2.log | cut -c1-300
