cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-g}
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python tools/phase_timing.py --gait --batch 1024 > gpurun_out/${TAG}_phase.log 2>&1
rc=$?; tail -7 gpurun_out/${TAG}_phase.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-host > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; python tools/summ.py gpurun_out/${TAG}_bench.log 2>/dev/null || tail -c 1500 gpurun_out/${TAG}_bench.log
