// race_f32.hip — race kernels and launchers for Real = float.  The step kernels of the physics
// modes are split over three translation units (race_f32.hip: PYB, PYB_DW — the benched ones and
// the dispatch; race_f32b.hip: DYN, PYB_GND; race_f32c.hip: PYB_DRAG, PYB_GND_DRAG_DW), so
// they compile in parallel.
#include "race_launch.h"

extern template ADRP_RACE_STEP_PH(float, ADRP_PHYS_DYN);
extern template ADRP_RACE_STEP_PH(float, ADRP_PHYS_PYB_GND);
extern template ADRP_RACE_STEP_PH(float, ADRP_PHYS_PYB_DRAG);
extern template ADRP_RACE_STEP_PH(float, ADRP_PHYS_PYB_GND_DRAG_DW);
template ADRP_RACE_STEP_PH(float, ADRP_PHYS_PYB);
template ADRP_RACE_STEP_PH(float, ADRP_PHYS_PYB_DW);

template int race_step<float>(adrp_t*, const float*, float*, float*, uint8_t*, uint8_t*, float*, hipStream_t);
template int race_reset<float>(adrp_t*, const uint8_t*, float*, hipStream_t);
template int race_command<float>(adrp_t*, const int32_t*, const double*, hipStream_t);
template int race_cmd_init<float>(adrp_t*, hipStream_t);

#ifdef ADRP_RACE_TIMING
ADRP_PHASE_READER(phase_read_race_f32)
#ifdef ADRP_RACE_GJK_STATS
ADRP_GJK_DUMP_READER(gjk_dump_read_f32)
#endif
ADRP_WAVE_READER(wave_read_race_f32)
#endif
