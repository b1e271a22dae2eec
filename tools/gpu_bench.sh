# bench (default legs) and its rocprofv3 kernel statistics
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 20 --no-cpu --legs 1500,imix,nat64,echo > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
