cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc $?"
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 bash tools/ab.sh gym_pybullet_adrp_amd/libadrp.so,ADRP_RACE_REFINE=1 gym_pybullet_adrp_amd/libadrp.so,ADRP_RACE_REFINE=0 2 --task race --level level0 --drones 2 --envs 2048 --policy example --steps 200 --warmup 20 > gpurun_out/ab_refine3p.log 2>&1; cat gpurun_out/ab_refine3p.log
timeout -k 10 300 bash tools/ab.sh gym_pybullet_adrp_amd/libadrp.so,ADRP_RACE_REFINE=1 gym_pybullet_adrp_amd/libadrp.so,ADRP_RACE_REFINE=0 2 --task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE --steps 200 --warmup 20 > gpurun_out/ab_refine4.log 2>&1; cat gpurun_out/ab_refine4.log
