# parity of the double-buffered kernel, then A/B against the round-1 kernel
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_frags.py tests/test_hostpath.py tests/test_max_frames.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/par_c.log 2>&1
for i in 1 2; do
  for lib in new old; do
    if [ $lib = old ]; then export XDPGPU_LIB=build/ab_7ebab66/libxdpgpu.so; else unset XDPGPU_LIB; fi
    echo "== $lib c2"; timeout -k 10 120 python -u tools/tune_rx.py --variants 64:0 --rounds 5
    echo "== $lib 1500"; timeout -k 10 120 python -u tools/tune_rx.py --frames 2097152 --size 1500 --variants 64:0 --rounds 5
    echo "== $lib imix"; timeout -k 10 120 python -u tools/tune_rx.py --frames 16777216 --kind 1 --seed 0x5EED0003 --variants 64:0 --rounds 5
  done
done
