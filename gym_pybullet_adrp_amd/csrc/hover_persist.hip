// hover_persist.hip — launcher of the persistent HoverAviary step (hover_persist.h; include/adrp.h
// adrp_persistent_*): the compiled-constant kernel for the reference default (CF2X at 240/30 Hz,
// PYB, RPM actions, 15-slot ring), the device-constant kernel with a runtime ring for every other
// physics mode and for ONE_D_RPM.  Both precisions; own translation unit (compiles in parallel).
#include "adrp_internal.h"
#include "hover_persist.h"

template <typename Real, int A>
static void launch_generic(const HoverArgs<Real>& a, PersistCtl* ctl, int physics, dim3 grid, hipStream_t s) {
    const dim3 blk(kStepBlock);
    switch (physics) {
        case ADRP_PHYS_PYB: hipLaunchKernelGGL((hover_persist_kernel<Real, ADRP_PHYS_PYB, A, 0, false>), grid, blk, 0, s, a, ctl); break;
        case ADRP_PHYS_DYN: hipLaunchKernelGGL((hover_persist_kernel<Real, ADRP_PHYS_DYN, A, 0, false>), grid, blk, 0, s, a, ctl); break;
        case ADRP_PHYS_PYB_GND: hipLaunchKernelGGL((hover_persist_kernel<Real, ADRP_PHYS_PYB_GND, A, 0, false>), grid, blk, 0, s, a, ctl); break;
        case ADRP_PHYS_PYB_DRAG: hipLaunchKernelGGL((hover_persist_kernel<Real, ADRP_PHYS_PYB_DRAG, A, 0, false>), grid, blk, 0, s, a, ctl); break;
        case ADRP_PHYS_PYB_DW: hipLaunchKernelGGL((hover_persist_kernel<Real, ADRP_PHYS_PYB_DW, A, 0, false>), grid, blk, 0, s, a, ctl); break;
        default: hipLaunchKernelGGL((hover_persist_kernel<Real, ADRP_PHYS_PYB_GND_DRAG_DW, A, 0, false>), grid, blk, 0, s, a, ctl); break;
    }
}

// which instantiation a handle's persistent step runs (adrp_handle_kernel_name in persistent mode)
bool hover_persist_def(const adrp_t* h) {
    return h->cf2x && h->B == 15 && h->A == 4 && h->cfg.physics == ADRP_PHYS_PYB;
}

template <typename Real>
int hover_persist_launch(adrp_t* h, const HoverArgs<Real>& a, void* ctl, hipStream_t s) {
    const dim3 grid((h->E + kStepBlock - 1) / kStepBlock);
    PersistCtl* c = (PersistCtl*)ctl;
    if (hover_persist_def(h))
        hipLaunchKernelGGL((hover_persist_kernel<Real, ADRP_PHYS_PYB, 4, 15, true>), grid, dim3(kStepBlock), 0, s, a, c);
    else if (h->A == 1)
        launch_generic<Real, 1>(a, c, h->cfg.physics, grid, s);
    else
        launch_generic<Real, 4>(a, c, h->cfg.physics, grid, s);
    HIPCHK(h, hipGetLastError());
    return ADRP_OK;
}

template int hover_persist_launch<float>(adrp_t*, const HoverArgs<float>&, void*, hipStream_t);
template int hover_persist_launch<double>(adrp_t*, const HoverArgs<double>&, void*, hipStream_t);
