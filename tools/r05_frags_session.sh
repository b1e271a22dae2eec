set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05_frags; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_frags.py > $O/tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -1 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python tools/frags_scale_probe.py 262144 > $O/new_$i.json 2>/dev/null || exit $?
XDPGPU_LIB=build/ab_HEAD/libxdpgpu.so timeout -k 10 200 python tools/frags_scale_probe.py 262144 > $O/old_$i.json 2>/dev/null || exit $?
done
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['ms_per_launch'], d['roofline_frac'], d['verdicts_ok'])")"; done
