# One box: the RX variants A/B (tools/tune_rx.py) and bench.py's config-2
# line back to back, so the bench number can be read against the A/B
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/tune_rx.py --variants ceil,64:0,64:2097152 --rounds 9 > gpurun_out/ab_b.log 2>&1 && cat gpurun_out/ab_b.log
timeout -k 10 300 python -u bench.py --no-cpu --no-secondary > gpurun_out/bench_b.log 2>&1 && tail -1 gpurun_out/bench_b.log | cut -c1-900
timeout -k 10 300 python -u tools/tune_rx.py --variants 64:0,64:2097152,ceil --rounds 9 > gpurun_out/ab_b2.log 2>&1 && cat gpurun_out/ab_b2.log
