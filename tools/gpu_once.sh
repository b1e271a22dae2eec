set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hints.py tests/test_abi.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_h.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|^FAILED|Error|error" gpurun_out/pytest_h.log | head -12
exit $rc
