# The tile stores' cache policy (XDP_VERDICT_AUX, XDP_REC_AUX, XDP_TUP4_AUX
# build knobs): parity of the in-tree build, then it against plain verdict
# stores (build/vpl) in alternating processes (tools/gpu_ab.sh)
set -u
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "imix or bulk or golden or udp4_64 or icmp" > gpurun_out/par_st.log 2>&1 || { tail -30 gpurun_out/par_st.log; exit 1; }
tail -1 gpurun_out/par_st.log
AB_B=build/vpl/libxdpgpu.so bash tools/gpu_ab.sh 2>&1 | grep -v amdgpu.ids | cut -c1-100
