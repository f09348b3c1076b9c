// race_f32.hip — race kernels and launchers for Real = float (own translation unit so
// the kernel instantiations compile in parallel)
#include "race_launch.h"

template int race_step<float>(adrp_t*, const float*, float*, float*, uint8_t*, uint8_t*, float*, hipStream_t);
template int race_reset<float>(adrp_t*, const uint8_t*, float*, hipStream_t);
template int race_command<float>(adrp_t*, const int32_t*, const double*, hipStream_t);
template int race_cmd_init<float>(adrp_t*, hipStream_t);

#ifdef ADRP_RACE_TIMING
ADRP_PHASE_READER(phase_read_race_f32)
ADRP_WAVE_READER(wave_read_race_f32)
#endif
