bash tools/gpu.sh evidence r5t && bash tools/gpu.sh prof r5t
