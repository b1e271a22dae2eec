#!/bin/bash
# SPDX-License-Identifier: GPL-2.0
# Host-code sanitizer build and run (AddressSanitizer + UndefinedBehavior-
# Sanitizer), CPU only, in this container: never on the GPU box.
#
# Builds into build/asan/ with clang's sanitizer runtime (one runtime for
# the whole process):
#   oracle/liboracle.so      the CPU restatement (test infrastructure)
#   csrc/libxdpgpu.so        the host C ABI, pool generator and nat64 state
#                            replay sanitized (-Xarch_host: the gfx950 code
#                            objects are the product's, unsanitized)
#   apps/xdpsock-gpu, af_xdp_user-gpu, xsk_probe   the front-ends and the
#                            AF_XDP ring code (apps/xsk.c, apps/rxapp.c)
# then runs the CPU suite (pytest -m "not gpu": oracle vs goldens, pool
# generator, nat64 state replay, the front-ends' pcap/pool/plumbing modes
# and, where the host allows AF_XDP, the live veth plumbing test) against
# those builds, with the runtime preloaded into python.
#   bash tools/asan.sh [pytest args...]     log: build/asan/pytest.log
# The reference builds its user code with gcc -O2 -g (lib/defines.mk:1) and
# has no sanitizer run.
set -eu
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/build/asan
rt=$(ls /opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
CLANG=/opt/rocm/llvm/bin/clang
HIPCC=/opt/rocm/bin/hipcc
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -shared-libsan"
HSAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer -Xarch_host -shared-libsan"
mkdir -p "$out/oracle" "$out/csrc" "$out/apps"

# oracle
( cd "$root/oracle" &&
  $CLANG -O1 -g $SAN -fPIC -shared -I../include -o "$out/oracle/liboracle.so" \
	xdp_oracle.c nat64_oracle.c synproxy_oracle.c cpu_leg.c -lpthread )

# libxdpgpu.so: the product's gfx950 objects, host C++ rebuilt sanitized
make -s -C "$root/bpf-examples_amd/csrc" >/dev/null
( cd "$root/bpf-examples_amd/csrc" &&
  for f in xdpgpu pool nat64_state; do
	$HIPCC -O1 -g -std=c++17 --offload-arch=gfx950 -fPIC $HSAN -I../../include -I. \
		-c $f.cpp -o "$out/csrc/$f.o"
  done &&
  $HIPCC -O1 -g --offload-arch=gfx950 -fPIC $HSAN -shared -o "$out/csrc/libxdpgpu.so" \
	xdp_rx.o nat64.o frags.o hints.o hostpath.o synproxy.o \
	"$out/csrc/xdpgpu.o" "$out/csrc/pool.o" "$out/csrc/nat64_state.o" -lpthread )

# front-ends
( cd "$root/bpf-examples_amd/apps" &&
  F="-O1 -g -Wall $SAN -I../../include"
  L="-L$out/csrc -Wl,-rpath,$out/csrc -Wl,-rpath-link,/opt/rocm/lib -lxdpgpu -lpthread"
  $CLANG $F -c xsk.c -o "$out/apps/xsk.o" &&
  $CLANG $F -c rxapp.c -o "$out/apps/rxapp.o" &&
  $CLANG $F -o "$out/apps/xsk_probe" xsk_probe.c "$out/apps/xsk.o" &&
  $CLANG $F -o "$out/apps/xdpsock-gpu" xdpsock_gpu.c "$out/apps/rxapp.o" "$out/apps/xsk.o" $L &&
  $CLANG $F -o "$out/apps/af_xdp_user-gpu" af_xdp_user_gpu.c "$out/apps/rxapp.o" \
	"$out/apps/xsk.o" $L )
echo "built $out"

cd "$root"
export XDPGPU_LIB=$out/csrc/libxdpgpu.so XDPGPU_ORACLE_LIB=$out/oracle/liboracle.so \
	XDPGPU_APPS=$out/apps
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:strict_string_checks=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
set +e
LD_PRELOAD=$rt python3 -m pytest tests -m "not gpu" -q -p no:cacheprovider "$@" \
	> "$out/pytest.log" 2>&1
rc=$?
tail -5 "$out/pytest.log"
n=$(grep -c "ERROR: AddressSanitizer\|runtime error:" "$out/pytest.log")
echo "sanitizer reports: $n (log $out/pytest.log)"
exit $rc
