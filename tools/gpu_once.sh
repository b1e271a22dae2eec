set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof64 -o run -- python3 bench.py --no-cpu --steps 10 --legs nat64 > gpurun_out/prof64.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof64.log; cat gpurun_out/prof64/run_kernel_stats.csv
