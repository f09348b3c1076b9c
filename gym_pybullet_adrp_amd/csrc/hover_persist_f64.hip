// hover_persist_f64.hip — the persistent HoverAviary step, Real = double (hover_persist_launch.h)
#include "hover_persist_launch.h"

template int hover_persist_launch<double>(adrp_t*, const HoverArgs<double>&, void*, hipStream_t);
