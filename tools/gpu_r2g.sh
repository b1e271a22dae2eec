# debug-build checks, GPU suite, RX variants, per-wave timeline
set -e
mkdir -p gpurun_out
XDPGPU_LIB=build/dbg/libxdpgpu.so timeout -k 10 300 python -u tools/dbg_golden.py > gpurun_out/dbg_g.log 2>&1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_frags.py tests/test_hostpath.py tests/test_max_frames.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/par_g.log 2>&1
bash tools/gpu_perf.sh
XDPGPU_LIB=build/stamps/libxdpgpu.so timeout -k 10 120 python -u tools/stamps.py
