set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05_gather6; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_nat64.py tests/test_nat64_inner.py tests/test_nat64_dyn.py > $O/tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for lib in csrc HEAD; do
  case $lib in csrc) L=;; HEAD) L=build/ab_HEAD/libxdpgpu.so;; esac
  XDPGPU_LIB=$L timeout -k 10 120 python tools/nat64_probe.py --reps 5 > $O/nat64_${lib}_$i.log 2>&1 || exit $?
  XDPGPU_LIB=$L timeout -k 10 120 python tools/nat64_probe.py --reps 5 --direction 1 > $O/nat64eg_${lib}_$i.log 2>&1 || exit $?
done
done
for f in $O/nat64*.log; do echo "$(basename $f .log) $(grep -o 'dir=.*' $f)"; done
