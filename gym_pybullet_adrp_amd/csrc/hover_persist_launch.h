// hover_persist_launch.h — launcher of the persistent HoverAviary step (hover_persist.h;
// include/adrp.h adrp_persistent_*), instantiated per precision by hover_persist_f32.hip /
// hover_persist_f64.hip.  The persistent kernel runs the row-store template of hover_step_kernel
// that a launched step of the same handle runs when its rows are not LDS-staged (E % 64 != 0):
// compiled-in constants for the reference drone at 240/30 Hz with the 15-slot ring, device
// constants and the runtime ring otherwise; RPM (A = 4) and ONE_D_RPM (A = 1) actions.
#pragma once

#include "adrp_internal.h"
#include "hover_persist.h"

template <typename Real, int A, int B, bool DEF, bool LINE>
static void launch_persist_ph(const HoverArgs<Real>& a, PersistCtl* ctl, int physics, dim3 grid, hipStream_t s) {
    const dim3 blk(kStepBlock);
    switch (physics) {
        case ADRP_PHYS_PYB: hipLaunchKernelGGL((hover_persist_kernel<Real, ADRP_PHYS_PYB, A, B, DEF, LINE>), grid, blk, 0, s, a, ctl); break;
        case ADRP_PHYS_DYN: hipLaunchKernelGGL((hover_persist_kernel<Real, ADRP_PHYS_DYN, A, B, DEF, LINE>), grid, blk, 0, s, a, ctl); break;
        case ADRP_PHYS_PYB_GND: hipLaunchKernelGGL((hover_persist_kernel<Real, ADRP_PHYS_PYB_GND, A, B, DEF, LINE>), grid, blk, 0, s, a, ctl); break;
        case ADRP_PHYS_PYB_DRAG: hipLaunchKernelGGL((hover_persist_kernel<Real, ADRP_PHYS_PYB_DRAG, A, B, DEF, LINE>), grid, blk, 0, s, a, ctl); break;
        case ADRP_PHYS_PYB_DW: hipLaunchKernelGGL((hover_persist_kernel<Real, ADRP_PHYS_PYB_DW, A, B, DEF, LINE>), grid, blk, 0, s, a, ctl); break;
        default: hipLaunchKernelGGL((hover_persist_kernel<Real, ADRP_PHYS_PYB_GND_DRAG_DW, A, B, DEF, LINE>), grid, blk, 0, s, a, ctl); break;
    }
}

template <typename Real>
int hover_persist_launch(adrp_t* h, const HoverArgs<Real>& a, void* ctl, hipStream_t s) {
    const dim3 grid((h->E + kStepBlock - 1) / kStepBlock);
    PersistCtl* c = (PersistCtl*)ctl;
    const int ph = h->cfg.physics;
    if (h->pline) {   // line mode (E * A <= 15): the action and its request tag in one 64-byte line
        if (h->cf2x && h->B == 15) {
            if (h->A == 1) launch_persist_ph<Real, 1, 15, true, true>(a, c, ph, grid, s);
            else launch_persist_ph<Real, 4, 15, true, true>(a, c, ph, grid, s);
        } else {
            if (h->A == 1) launch_persist_ph<Real, 1, 0, false, true>(a, c, ph, grid, s);
            else launch_persist_ph<Real, 4, 0, false, true>(a, c, ph, grid, s);
        }
    } else if (h->cf2x && h->B == 15) {
        if (h->A == 1) launch_persist_ph<Real, 1, 15, true, false>(a, c, ph, grid, s);
        else launch_persist_ph<Real, 4, 15, true, false>(a, c, ph, grid, s);
    } else {
        if (h->A == 1) launch_persist_ph<Real, 1, 0, false, false>(a, c, ph, grid, s);
        else launch_persist_ph<Real, 4, 0, false, false>(a, c, ph, grid, s);
    }
    HIPCHK(h, hipGetLastError());
    return ADRP_OK;
}
