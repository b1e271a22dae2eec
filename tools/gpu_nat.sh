set -e
for r in 1 2; do
for lib in bpf-examples_amd/csrc/libxdpgpu.so build/ab_nat_nt/libxdpgpu.so; do
  echo "== $lib"
  XDPGPU_LIB=$lib timeout -k 10 100 python -u tools/nat64_probe.py
  XDPGPU_LIB=$lib timeout -k 10 100 python -u tools/nat64_probe.py --direction 1
done
done
