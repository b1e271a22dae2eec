set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05_gather7; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hostpath.py > $O/tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/e2e_probe.py > $O/e2e.jsonl 2>&1; echo e2e rc=$?; grep mode $O/e2e.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof -o e2e -- python3 tools/e2e_probe.py --gather-only --batches 16 > $O/prof.log 2>&1; echo prof rc=$?
