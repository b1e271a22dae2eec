set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|^FAILED" gpurun_out/pytest.log | head -8
[ $rc -eq 0 ] || exit $rc
s=$(date +%s); timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 3; echo "bench $(( $(date +%s) - s )) s"
python3 -c "
import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'])
for k in ('secondary_1500B','config3_imix','config4_nat64','multibuffer_9000B'): print(k, {x: d[k].get(x) for x in ('mpps','ms_per_launch','kernel_ms','verdicts_ok','actions_ok')})
"
for lib in build/ab_HEAD/libxdpgpu.so bpf-examples_amd/csrc/libxdpgpu.so build/ab_HEAD/libxdpgpu.so bpf-examples_amd/csrc/libxdpgpu.so; do
  XDPGPU_LIB=$lib timeout -k 10 300 python3 tools/tune_rx.py --variants 64:0 --rounds 7 > gpurun_out/t64.log 2>&1 || exit 3; echo "$lib $(grep -v amdgpu.ids gpurun_out/t64.log | cut -c1-60)"
done
