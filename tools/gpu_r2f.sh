# GPU suite, then the RX variants
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_frags.py tests/test_hostpath.py tests/test_max_frames.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/par_f.log 2>&1
bash tools/gpu_perf.sh
