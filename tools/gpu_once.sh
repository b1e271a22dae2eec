set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  echo "== new $i"; timeout -k 10 120 python -u tools/frags_probe.py --reps 5
  echo "== old $i"; XDPGPU_LIB=build/ab_HEAD/libxdpgpu.so timeout -k 10 120 python -u tools/frags_probe.py --reps 5
done > gpurun_out/frag_ab.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_frags.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/frag_par.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fragnew -o run -- python3 tools/frags_probe.py --reps 5 > gpurun_out/prof_fragnew.log 2>&1
