mkdir -p gpurun_out/r5d && \
TESTS="tests/test_persistent_gpu.py" bash tools/gpu.sh check r5d ; \
ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devc.so RACE_PRECISION=fp64 timeout -k 10 200 python tools/race_phases.py level3 4 PYB_DW COMPETE 4096 > gpurun_out/r5d/ctrl_phases_c4_fp64.log 2>&1 && tail -1 gpurun_out/r5d/ctrl_phases_c4_fp64.log && \
ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devc.so RACE_PRECISION=fp64 timeout -k 10 200 python tools/race_phases.py level0 2 PYB COMPARE 2048 > gpurun_out/r5d/ctrl_phases_c3_fp64.log 2>&1 && tail -1 gpurun_out/r5d/ctrl_phases_c3_fp64.log && \
ADRP_LIB=gym_pybullet_adrp_amd/libadrp_devc.so RACE_PRECISION=fp32 timeout -k 10 200 python tools/race_phases.py level3 4 PYB_DW COMPETE 4096 > gpurun_out/r5d/ctrl_phases_c4_fp32.log 2>&1 && tail -1 gpurun_out/r5d/ctrl_phases_c4_fp32.log
