# A tail change against the committed tree's build (tools/ab_build.sh HEAD):
# parity of the pools, bulk lengths and golden fixtures, then alternating
# processes (tools/gpu_ab.sh: IMIX, 1500 B, config 2)
set -u
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_max_frames.py -m gpu -x -q --timeout 200 --timeout-method thread -k "imix or bulk or golden or 1500 or max or icmp" > gpurun_out/par_t6.log 2>&1 || { tail -30 gpurun_out/par_t6.log; exit 1; }
tail -1 gpurun_out/par_t6.log
AB_B=build/ab_HEAD/libxdpgpu.so bash tools/gpu_ab.sh 2>&1 | grep -v amdgpu.ids | cut -c1-110
