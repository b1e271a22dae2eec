set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|^FAILED" gpurun_out/pytest.log | head -8
exit $rc
