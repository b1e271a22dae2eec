set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_max_frames.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/max.log 2>&1
