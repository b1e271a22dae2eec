# A/B of xdp_rx_db_kernel's shared tiles (cfg.tune bits 21-22) and tile
# orders (bits 19-20): parity of the variants on the pools, then config 2
# and config 3 timings in one process each
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/par_steal.log 2>&1 || { tail -30 gpurun_out/par_steal.log; exit 1; }
tail -3 gpurun_out/par_steal.log
timeout -k 10 300 python -u tools/tune_rx.py --variants ceil,64:2097152,64:6291456,64:10485760,64:14680064,64:8388608 --rounds 9 > gpurun_out/ab_c2.log 2>&1 && cat gpurun_out/ab_c2.log
timeout -k 10 300 python -u tools/tune_rx.py --variants 64:2097152,64:6291456,64:10485760,64:8388608 --rounds 5 --frames 16777216 --kind 1 --seed 0x5EED0003 --fmt 2 > gpurun_out/ab_c3.log 2>&1 && cat gpurun_out/ab_c3.log
XDPGPU_LIB=build/stamps/libxdpgpu.so timeout -k 10 120 python -u tools/stamps.py 16777216 8388608 > gpurun_out/st2q.log 2>&1 && cat gpurun_out/st2q.log; XDPGPU_LIB=build/stamps/libxdpgpu.so timeout -k 10 120 python -u tools/stamps.py 16777216 10485760 > gpurun_out/st2s.log 2>&1 && cat gpurun_out/st2s.log
