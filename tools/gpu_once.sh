set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|^FAILED|Error" gpurun_out/pytest.log | head -8
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
for lib in build/ab_HEAD/libxdpgpu.so bpf-examples_amd/csrc/libxdpgpu.so; do
XDPGPU_LIB=$lib timeout -k 10 300 python3 tools/tune_rx.py --variants 64:0 --rounds 7 > gpurun_out/t64.log 2>&1 || exit 3; echo "$lib $(grep -v amdgpu.ids gpurun_out/t64.log | cut -c1-50,120-300)"
done
done
