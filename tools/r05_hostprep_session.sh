set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05_hostprep; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hostpath.py tests/test_gpu_parity.py -k "ring or host or scattered or chunked or gather or submit" > $O/tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -1 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python tools/e2e_probe.py --packed --frames 16777216 > $O/new_$i.json 2>/dev/null || exit $?
XDPGPU_LIB=build/ab_HEAD/libxdpgpu.so timeout -k 10 200 python tools/e2e_probe.py --packed --frames 16777216 > $O/old_$i.json 2>/dev/null || exit $?
done
for f in $O/*.json; do echo "$f $(python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['mpps'], d['pcie_frac'], d['submit_host_ms'], d['verdicts_ok'])")"; done
