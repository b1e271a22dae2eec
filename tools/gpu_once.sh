set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nat64.py tests/test_apps.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_nat64.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|^FAILED|Error" gpurun_out/pytest_nat64.log | head -12
[ $rc -eq 0 ] || exit $rc
for lib in build/ab_HEAD/libxdpgpu.so bpf-examples_amd/csrc/libxdpgpu.so; do
for args in "--direction 0" "--direction 1" "--direction 1 --headroom 32"; do
  XDPGPU_LIB=$lib timeout -k 10 300 python3 tools/nat64_probe.py $args > gpurun_out/n64.log 2>&1 || exit 3; echo "$lib $args: $(grep -v amdgpu.ids gpurun_out/n64.log | cut -c1-80)"
done
done
