set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_frags.py tests/test_hostpath.py tests/test_max_frames.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/par.log 2>&1
echo "== c2"; timeout -k 10 120 python -u tools/tune_rx.py --variants ceil,64:0,64:32768 --rounds 7
echo "== 1500"; timeout -k 10 120 python -u tools/tune_rx.py --frames 2097152 --size 1500 --variants 64:0,64:32768 --rounds 5
echo "== imix"; timeout -k 10 120 python -u tools/tune_rx.py --frames 16777216 --kind 1 --seed 0x5EED0003 --variants 64:0,64:32768 --rounds 5
