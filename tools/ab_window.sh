set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04_s23
for r in 1 2; do
  for w in 64 0; do
    timeout -k 10 240 python3 bench.py --no-cpu --no-e2e --legs echo,imix,1500 --steps 10 --warmup 3 --window $w > gpurun_out/r04_s23/bench_w${w}_$r.log 2>&1 || exit $?
  done
done
