# A/B of xdp_rx_db_kernel's shared tiles (cfg.tune bits 21-23): parity of
# every variant on the pools and the golden fixtures on the bounds-checked
# build, then config 2 and config 3 timings in one process each
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/par_steal.log 2>&1 || { tail -30 gpurun_out/par_steal.log; exit 1; }
tail -2 gpurun_out/par_steal.log
XDPGPU_LIB=build/dbg/libxdpgpu.so timeout -k 10 300 python -u tools/dbg_golden.py > gpurun_out/dbg_g.log 2>&1 || { tail -20 gpurun_out/dbg_g.log; exit 1; }
cat gpurun_out/dbg_g.log
timeout -k 10 300 python -u tools/tune_rx.py --variants ceil,64:2097152,64:0,64:16777216,64:14680064,64:31457280 --rounds 15 > gpurun_out/ab_c2.log 2>&1 && cat gpurun_out/ab_c2.log
timeout -k 10 300 python -u tools/tune_rx.py --variants 64:0,64:2097152,64:16777216 --rounds 5 --frames 16777216 --kind 1 --seed 0x5EED0003 --fmt 2 > gpurun_out/ab_c3.log 2>&1 && cat gpurun_out/ab_c3.log
