set -u
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "imix or bulk or golden" > gpurun_out/par_t6.log 2>&1 || { tail -30 gpurun_out/par_t6.log; exit 1; }
tail -1 gpurun_out/par_t6.log
AB_B=build/ab_HEAD/libxdpgpu.so bash tools/gpu_ab.sh 2>&1 | grep -v amdgpu.ids | cut -c1-140
