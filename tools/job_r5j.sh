L=gym_pybullet_adrp_amd/libadrp.so
O=gpurun_out/r5j; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_reset_images_gpu.py > $O/img_tests.log 2>&1; rc=$?; tail -5 $O/img_tests.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -ge 124 ] && exit $rc
R4="--task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE --steps 1000 --warmup 50"
BENCH_ARGS="$R4" bash tools/gpu.sh ab r5j_ab4 2 $L $L,ADRP_RESET_IMAGES=0 && \
BENCH_ARGS="$R4 --precision fp32" bash tools/gpu.sh ab r5j_ab4f 2 $L $L,ADRP_RESET_IMAGES=0 && \
BENCH_ARGS="--task race --level level0 --drones 2 --envs 2048 --physics PYB --racemode COMPARE --steps 1000 --warmup 50 --policy example" bash tools/gpu.sh ab r5j_ab3p 2 $L $L,ADRP_RESET_IMAGES=0 && \
bash tools/gpu.sh prof r5j
