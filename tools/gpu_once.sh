set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|^FAILED|Error" gpurun_out/pytest.log | head -8
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
timeout -k 10 300 python3 tools/tune_rx.py --variants 64:0,64:2048 --rounds 5 > gpurun_out/t64.log 2>&1 || exit 3; grep -v amdgpu.ids gpurun_out/t64.log | cut -c1-50,120-300
timeout -k 10 300 python3 tools/tune_rx.py --variants 64:0,64:2048 --rounds 5 --frames 2097152 --size 1500 > gpurun_out/t15.log 2>&1 || exit 3; grep -v amdgpu.ids gpurun_out/t15.log | cut -c1-50,120-300
timeout -k 10 300 python3 tools/tune_rx.py --variants 64:0,64:2048 --rounds 3 --kind 1 --seed 0x5EED0003 > gpurun_out/timix.log 2>&1 || exit 3; grep -v amdgpu.ids gpurun_out/timix.log | cut -c1-50,120-300
done
