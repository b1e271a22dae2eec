set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06_base
mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-e2e --no-secondary > $O/bench_plain.json 2> $O/bench_plain.log || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-e2e --no-secondary > $O/bench_prof.json 2> $O/bench_prof.log || exit $?
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 tools/trace_gaps.py "$f" --json $O/gaps.json > $O/gaps.txt
cat $O/bench_plain.json $O/bench_prof.json
tail -50 $O/gaps.txt
