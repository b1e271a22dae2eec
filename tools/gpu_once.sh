set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "1024" > gpurun_out/ab_par.log 2>&1
timeout -k 10 200 python -u tools/tune_rx.py --frames 2097152 --size 1500 --variants 64:0,64:1024 --rounds 9 > gpurun_out/ab_1500.log 2>&1
timeout -k 10 200 python -u tools/tune_rx.py --frames 16777216 --kind 1 --variants 64:0,64:1024 --rounds 9 > gpurun_out/ab_imix.log 2>&1
