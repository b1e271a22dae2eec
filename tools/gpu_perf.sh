# RX variants: config 2 (64 B), 1500 B and IMIX; 64:0 = one double-buffered
# launch, 64:32768 = the three-kernel path, 65536/131072 = its diagnostics
set -e
echo "== c2"; timeout -k 10 120 python -u tools/tune_rx.py --variants ceil,64:0,64:65536,64:131072,64:32768 --rounds 7
echo "== 1500"; timeout -k 10 120 python -u tools/tune_rx.py --frames 2097152 --size 1500 --variants 64:0,64:32768 --rounds 5
echo "== imix"; timeout -k 10 120 python -u tools/tune_rx.py --frames 16777216 --kind 1 --seed 0x5EED0003 --variants 64:0,64:32768 --rounds 5
