// race_f64c.hip — fp64 race step kernels of PYB_DRAG and PYB_GND_DRAG_DW (see race_f64.hip)
#include "race_launch.h"

#ifndef ADRP_DEV_FAST
template ADRP_RACE_STEP_PH(double, ADRP_PHYS_PYB_DRAG);
template ADRP_RACE_STEP_PH(double, ADRP_PHYS_PYB_GND_DRAG_DW);
#endif

#ifdef ADRP_RACE_TIMING
ADRP_PHASE_READER(phase_read_race_f64c)
#endif
