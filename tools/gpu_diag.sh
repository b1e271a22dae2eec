# one-off diagnostic: kernels serialized, each launch's error reported at
# the launch that caused it
set -e
mkdir -p gpurun_out
export AMD_SERIALIZE_KERNEL=3
timeout -k 10 300 python -u -m pytest tests/test_max_frames.py -x -s -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/diag_max.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_hostpath.py -x -s -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/diag_hp.log 2>&1
