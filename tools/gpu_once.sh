set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_frags.py tests/test_apps.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_frags.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|^FAILED|Error|error" gpurun_out/pytest_frags.log | head -12
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pf -o run -- python3 $GRAFT_REPO_ROOT/tools/frags_probe.py > $GRAFT_REPO_ROOT/gpurun_out/pf.log 2>&1 || exit 3
grep -v "amdgpu.ids\|^W20\|^E20" $GRAFT_REPO_ROOT/gpurun_out/pf.log | tail -3
python3 -c "
import csv
for r in csv.DictReader(open('$GRAFT_REPO_ROOT/gpurun_out/pf/run_kernel_stats.csv')):
    if 'frag' in r['Name'] or 'xdp_rx' in r['Name']: print(r['Name'][:70], r['Calls'], r['AverageNs'])
"
