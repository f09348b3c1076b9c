bash tools/gpu.sh check r5s
