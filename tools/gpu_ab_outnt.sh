# Non-temporal nat64 action/descriptor stores and bulk-pass verdicts
# (build/outnt) against the in-tree build, alternating processes
set -u
B=build/outnt/libxdpgpu.so
A=bpf-examples_amd/csrc/libxdpgpu.so
XDPGPU_LIB=$B timeout -k 10 300 python -u -m pytest tests/test_nat64.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "gpu_pool or imix or bulk" > gpurun_out/par_outnt.log 2>&1 || { tail -30 gpurun_out/par_outnt.log; exit 1; }
tail -1 gpurun_out/par_outnt.log
for r in 1 2 3; do for lib in $A $B; do
  echo "== $lib"
  XDPGPU_LIB=$lib timeout -k 10 120 python -u tools/nat64_probe.py --reps 10 2>&1 | grep -v amdgpu.ids | cut -c1-100 || exit 1
  XDPGPU_LIB=$lib timeout -k 10 120 python -u tools/tune_rx.py --variants 64:0 --rounds 3 --frames 16777216 --kind 1 --seed 0x5EED0003 --fmt 2 2>&1 | grep -v amdgpu.ids | cut -c1-100 || exit 1
done; done
