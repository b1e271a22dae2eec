set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_apps.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
for b in 65536 1048576; do
timeout -k 10 120 bpf-examples_amd/apps/xdpsock-gpu --pool 16777216 --pool-kind udp4 -b $b -C 67108864 --json -Q > gpurun_out/cli.log 2>&1; rc=$?; echo "cli b=$b rc=$rc"; tail -1 gpurun_out/cli.log
[ $rc -eq 0 ] || exit $rc
done
