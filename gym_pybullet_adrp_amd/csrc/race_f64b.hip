// race_f64b.hip — fp64 race step kernels of DYN and PYB_GND (see race_f64.hip)
#include "race_launch.h"

#ifndef ADRP_DEV_FAST
template ADRP_RACE_STEP_PH(double, ADRP_PHYS_DYN);
template ADRP_RACE_STEP_PH(double, ADRP_PHYS_PYB_GND);
#endif

#ifdef ADRP_RACE_TIMING
ADRP_PHASE_READER(phase_read_race_f64b)
#endif
