// hover_f64.hip — hover kernels and launchers for Real = double (own translation unit so
// the kernel instantiations compile in parallel)
#include "hover_launch.h"

template int hover_step<double>(adrp_t*, const float*, float*, float*, uint8_t*, uint8_t*, float*, hipStream_t);
template int hover_reset<double>(adrp_t*, const uint8_t*, float*, hipStream_t);

#ifdef ADRP_RACE_TIMING
ADRP_PHASE_READER(phase_read_hover_f64)
#endif
