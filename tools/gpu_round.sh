#!/bin/bash
# One GPU session: parity tests, smoke, benches (hover default + race configs 3/4), kernel-trace
# profiles, HBM PMC passes (hover E = 4096 and 2^20, race config 4).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r1}"
PHASE="${2:-all}"     # test | prof | all (one gpurun call is capped at 1200 s: run test and prof separately)
PROF="cd /tmp && export TMPDIR=/tmp && rocprofv3"
RACE4="level3 4 PYB_DW COMPETE 4096"
T=(
  "pytest_gpu|600|cd $R && python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"
  "smoke|200|cd $R && python -c 'import __graft_entry__ as g; g.smoke()'"
  "bench|300|cd $R && python bench.py"
  "bench_race3|300|cd $R && python bench.py --task race --level level0 --drones 2 --envs 2048 --steps 300 --warmup 30"
  "bench_race4|300|cd $R && python bench.py --task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE --steps 200 --warmup 20"
)
P=(
  "prof_$TAG|300|$PROF --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o bench -- python3 $R/bench.py --steps 2000 --no-cpu-baseline"
  "profrace_$TAG|300|$PROF --kernel-trace --stats --output-format csv -d $R/gpurun_out/profrace_$TAG -o bench -- python3 $R/bench.py --task race --level level3 --drones 4 --envs 4096 --physics PYB_DW --racemode COMPETE --steps 200 --warmup 20 --no-cpu-baseline"
  "pmcf4k|200|$PROF --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf4k_$TAG -o p -- python3 $R/tools/pmc_steps.py 4096 200 fp32 $R"
  "pmcw4k|200|$PROF --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw4k_$TAG -o p -- python3 $R/tools/pmc_steps.py 4096 200 fp32 $R"
  "pmcf1m|200|$PROF --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf1m_$TAG -o p -- python3 $R/tools/pmc_steps.py 1048576 40 fp32 $R"
  "pmcw1m|200|$PROF --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcw1m_$TAG -o p -- python3 $R/tools/pmc_steps.py 1048576 40 fp32 $R"
  "pmcfr4|200|$PROF --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcfr4_$TAG -o p -- python3 $R/tools/pmc_race_steps.py $RACE4 40 $R"
  "pmcwr4|200|$PROF --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcwr4_$TAG -o p -- python3 $R/tools/pmc_race_steps.py $RACE4 40 $R"
)
case "$PHASE" in
  test) exec "$R/tools/gpu_steps.sh" "${T[@]}" ;;
  prof) exec "$R/tools/gpu_steps.sh" "${P[@]}" ;;
  *) exec "$R/tools/gpu_steps.sh" "${T[@]}" "${P[@]}" ;;
esac
