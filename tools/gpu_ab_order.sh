# A/B of xdp_rx_db_kernel's tile orders (cfg.tune bits 19-20): parity of the
# variants, then config 2 and config 3 timings in one process each
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "524288 or 1048576 or 1572864" > gpurun_out/par_order.log 2>&1 || { tail -30 gpurun_out/par_order.log; exit 1; }
tail -3 gpurun_out/par_order.log
timeout -k 10 300 python -u tools/tune_rx.py --variants ceil,64:0,64:1048576,64:1572864 --rounds 9 > gpurun_out/ab_c2.log 2>&1 && cat gpurun_out/ab_c2.log
timeout -k 10 300 python -u tools/tune_rx.py --variants 64:0,64:1048576,64:1572864 --rounds 5 --frames 16777216 --kind 1 --seed 0x5EED0003 --fmt 2 > gpurun_out/ab_c3.log 2>&1 && cat gpurun_out/ab_c3.log
