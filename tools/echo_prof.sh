set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05_echo_prof; mkdir -p $O
export TMPDIR=/tmp
for d in 0 64 127; do
STAMPS_SIZE=128 STAMPS_ECHO_PPM=200000 STAMPS_WINDOW=0 STAMPS_REPS=3 XDPGPU_LIB=build/s_d$d/libxdpgpu.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/d$d -o s -- python3 tools/stamps.py 8388608 0 0 1 > $O/d$d.json 2> $O/d$d.err || exit $?
done
