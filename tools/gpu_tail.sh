# tail A/B on IMIX (NET) and 1500 B, same box, interleaved twice; checks
set -e
XDPGPU_LIB=build/dbg/libxdpgpu.so timeout -k 10 300 python -u tools/dbg_golden.py > gpurun_out/dbg_t.log 2>&1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_frags.py tests/test_hostpath.py tests/test_max_frames.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/par_t.log 2>&1
for r in 1 2; do
for lib in bpf-examples_amd/csrc/libxdpgpu.so build/ab_prev/libxdpgpu.so; do
  echo "== $lib"
  XDPGPU_LIB=$lib timeout -k 10 100 python -u tools/tune_rx.py --frames 16777216 --kind 1 --seed 0x5EED0003 --variants 64:0 --rounds 3 --fmt 2
done
done
XDPGPU_LIB=build/stamps/libxdpgpu.so timeout -k 10 100 python -u tools/stamps.py 16777216 0 1 2
