# debug-build bounds checks on golden / IMIX / max frames, then the GPU
# suite with per-test drains (names each test)
set -e
mkdir -p gpurun_out
XDPGPU_LIB=build/dbg/libxdpgpu.so timeout -k 10 300 python -u tools/dbg_golden.py > gpurun_out/dbg_e.log 2>&1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_frags.py tests/test_hostpath.py tests/test_max_frames.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/par_e.log 2>&1
