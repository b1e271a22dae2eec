set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_frags.py tests/test_max_frames.py tests/test_hostpath.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/par_icmp.log 2>&1 || { tail -30 gpurun_out/par_icmp.log; exit 1; }
tail -2 gpurun_out/par_icmp.log
XDPGPU_LIB=build/dbg/libxdpgpu.so timeout -k 10 300 python -u tools/dbg_golden.py > gpurun_out/dbg_g.log 2>&1 || { tail -20 gpurun_out/dbg_g.log; exit 1; }
cat gpurun_out/dbg_g.log
timeout -k 10 300 python -u tools/tune_rx.py --variants 64:0 --rounds 5 --frames 16777216 --kind 1 --seed 0x5EED0003 --fmt 2 > gpurun_out/ab_c3.log 2>&1 && cat gpurun_out/ab_c3.log
