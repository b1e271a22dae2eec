# live AF_XDP on the GPU box: plumbing probe, then config 1 through the GPU
mkdir -p gpurun_out
id > gpurun_out/live_id.txt
timeout -k 5 60 ./bpf-examples_amd/apps/xsk_probe --caps > gpurun_out/live_caps.json 2>&1; timeout -k 5 60 ./bpf-examples_amd/apps/xsk_probe --frames 4096 > gpurun_out/live_probe.json 2>&1
echo "probe rc=$?" >> gpurun_out/live_probe.json
timeout -k 5 60 ./bpf-examples_amd/apps/xdpsock-gpu -i xgl0 --veth xgl1 --inject 20000 --pool-kind udp4 -s 64 -S -r -Q --json -C 20000 --verdicts gpurun_out/live_v.bin > gpurun_out/live_run.json 2>&1
echo "run rc=$?" >> gpurun_out/live_run.json
exit 0
