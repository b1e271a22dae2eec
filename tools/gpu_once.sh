set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_frags.py tests/test_apps.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_frags.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|^FAILED|Error|error" gpurun_out/pytest_frags.log | head -12
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_fr -o run -- python3 $GRAFT_REPO_ROOT/tools/frags_probe.py > $GRAFT_REPO_ROOT/gpurun_out/prof_fr.log 2>&1 || exit 3
grep -v "amdgpu.ids\|^W20\|^E20" $GRAFT_REPO_ROOT/gpurun_out/prof_fr.log | tail -3
cut -d, -f1-4 $GRAFT_REPO_ROOT/gpurun_out/prof_fr/run_kernel_stats.csv | cut -c1-120
