# nat64 fast kernel diagnostics (cfg.tune bits 12-13: no map probe / no
# frame stores), alternating processes, then the stride probe
set -u
T=${T:-"0 0x1000 0x2000 0x3000"}
for r in 1 2; do for t in $T; do
timeout -k 10 120 python -u tools/nat64_probe.py --reps 10 --tune $t --direction 0 2>&1 | grep -v amdgpu.ids || exit 1
done; done
timeout -k 10 120 tools/hbm_probe stride
