# nat64 fast kernel's shared tiles (cfg.tune bit 14 turns them off): the
# nat64 GPU tests, then alternating processes per variant and direction
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_nat64.py tests/test_nat64_dyn.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/par_nat.log 2>&1 || { tail -30 gpurun_out/par_nat.log; exit 1; }
tail -2 gpurun_out/par_nat.log
for r in 1 2 3; do
  for t in 0 0x4000; do
    for d in 0 1; do
      timeout -k 10 120 python -u tools/nat64_probe.py --reps 10 --tune $t --direction $d 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
