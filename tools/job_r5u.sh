bash tools/gpu.sh pmc r5t alg fp64 fp32
