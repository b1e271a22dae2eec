# Non-temporal descriptor DMA in the tile loop (build/dnt) against the
# in-tree build: golden/pool parity of the variant, then alternating
# processes (tools/gpu_ab.sh)
set -u
XDPGPU_LIB=build/dnt/libxdpgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "udp4_64 or golden" > gpurun_out/par_dnt.log 2>&1 || { tail -30 gpurun_out/par_dnt.log; exit 1; }
tail -1 gpurun_out/par_dnt.log
AB_B=build/dnt/libxdpgpu.so bash tools/gpu_ab.sh 2>&1 | grep -v amdgpu.ids | cut -c1-100
