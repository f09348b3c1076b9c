O=gpurun_out/r5h; mkdir -p $O
timeout -k 10 240 python tools/persist_probe.py 5000 1500 > $O/probe_fence.json 2> $O/probe_fence.err && \
ADRP_PERSIST_SYSST=1 timeout -k 10 240 python tools/persist_probe.py 5000 1500 > $O/probe_sysst.json 2> $O/probe_sysst.err && \
cat $O/probe_fence.json $O/probe_sysst.json && \
bash tools/gpu.sh phases r5h gym_pybullet_adrp_amd/libadrp_devt.so
