// race_f64.hip — race kernels and launchers for Real = double.  The step kernels of the physics
// modes are split over three translation units as in fp32 (race_f64.hip: PYB, PYB_DW — the benched
// ones and the dispatch; race_f64b.hip: DYN, PYB_GND; race_f64c.hip: PYB_DRAG, PYB_GND_DRAG_DW).
#include "race_launch.h"

extern template ADRP_RACE_STEP_PH(double, ADRP_PHYS_DYN);
extern template ADRP_RACE_STEP_PH(double, ADRP_PHYS_PYB_GND);
extern template ADRP_RACE_STEP_PH(double, ADRP_PHYS_PYB_DRAG);
extern template ADRP_RACE_STEP_PH(double, ADRP_PHYS_PYB_GND_DRAG_DW);
template ADRP_RACE_STEP_PH(double, ADRP_PHYS_PYB);
template ADRP_RACE_STEP_PH(double, ADRP_PHYS_PYB_DW);

template int race_step<double>(adrp_t*, const float*, float*, float*, uint8_t*, uint8_t*, float*, hipStream_t);
template int race_reset<double>(adrp_t*, const uint8_t*, float*, hipStream_t);
template int race_command<double>(adrp_t*, const int32_t*, const double*, hipStream_t);
template int race_cmd_init<double>(adrp_t*, hipStream_t);

#ifdef ADRP_RACE_TIMING
ADRP_PHASE_READER(phase_read_race_f64)
#ifdef ADRP_RACE_GJK_STATS
ADRP_GJK_DUMP_READER(gjk_dump_read_f64)
#endif
ADRP_WAVE_READER(wave_read_race_f64)
#endif
