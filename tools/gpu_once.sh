set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nat64.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
for t in 0 0x1000 0x2000; do
timeout -k 10 120 python3 tools/nat64_probe.py --tune $t > gpurun_out/probe.log 2>&1; rc=$?; tail -1 gpurun_out/probe.log
[ $rc -eq 0 ] || exit $rc
done
