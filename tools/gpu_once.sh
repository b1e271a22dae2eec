set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
OLD=build/ab_01e11cb/libxdpgpu.so
for rep in 1 2; do
for lib in $OLD bpf-examples_amd/csrc/libxdpgpu.so; do
  echo "== $lib"
  XDPGPU_LIB=$lib timeout -k 10 300 python3 tools/tune_rx.py --variants ceil,64:0 --rounds 5 > gpurun_out/t64.log 2>&1 || exit 3; grep -v amdgpu.ids gpurun_out/t64.log
  XDPGPU_LIB=$lib timeout -k 10 300 python3 tools/tune_rx.py --variants 64:0 --rounds 5 --frames 2097152 --size 1500 > gpurun_out/t1500.log 2>&1 || exit 3; grep -v amdgpu.ids gpurun_out/t1500.log
done
done
