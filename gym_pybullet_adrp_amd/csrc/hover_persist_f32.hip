// hover_persist_f32.hip — the persistent HoverAviary step, Real = float (hover_persist_launch.h)
#include "hover_persist_launch.h"

template int hover_persist_launch<float>(adrp_t*, const HoverArgs<float>&, void*, hipStream_t);
