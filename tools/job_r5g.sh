TESTS="tests/test_persistent_gpu.py tests/test_sharding_gpu.py" bash tools/gpu.sh check r5g && bash tools/gpu.sh prof r5g
