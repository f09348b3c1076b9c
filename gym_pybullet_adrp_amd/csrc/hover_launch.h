// hover_launch.h — HoverAviary step/reset launchers (instantiated by hover_f32.hip / hover_f64.hip)
#pragma once

#include "adrp_internal.h"

// ---------------------------------------------------------------------------------------------
// launch dispatch
// ---------------------------------------------------------------------------------------------

// launch with optional start/stop events recorded by the dispatch itself
template <typename K, typename Real>
static void launch(K kernel, dim3 grid, dim3 blk, hipStream_t s, const HoverArgs<Real>& a, adrp_t* h) {
    HoverTail<Real> t;
    memset(&t, 0, sizeof t);
    t.c = a.c; t.r = a.r; t.term = a.term; t.trunc = a.trunc; t.tobs = a.tobs; t.contact_count = a.contact_count;
    t.seed = a.seed; t.env_offset = a.env_offset; t.B = a.B; t.D = a.D; t.autoreset = a.autoreset;
    if (h->prof_n < h->prof_cap) {
        hipExtLaunchKernelGGL(kernel, grid, blk, 0, s, h->ev_start[h->prof_n], h->ev_stop[h->prof_n], 0,
                              a.f, a.ring, a.ist, a.act, a.obs, a.rew, a.E, t);
        ++h->prof_n;
    } else {
        hipLaunchKernelGGL(kernel, grid, blk, 0, s, a.f, a.ring, a.ist, a.act, a.obs, a.rew, a.E, t);
    }
}

template <typename Real, int A, int B, bool DEF, bool STG = false, int CTL = 0, bool HELP = false>
static void launch_step_ph(const HoverArgs<Real>& a, int physics, dim3 grid, hipStream_t s, adrp_t* h) {
    const dim3 blk(HELP ? (1 + help_waves<Real>()) * kBlock : kBlock);   // HELP: + the reset helper (and angle helper) waves
    switch (physics) {
        case ADRP_PHYS_PYB: launch(hover_step_kernel<Real, ADRP_PHYS_PYB, A, B, DEF, STG, CTL, HELP>, grid, blk, s, a, h); break;
        case ADRP_PHYS_DYN: launch(hover_step_kernel<Real, ADRP_PHYS_DYN, A, B, DEF, STG, CTL, HELP>, grid, blk, s, a, h); break;
        case ADRP_PHYS_PYB_GND: launch(hover_step_kernel<Real, ADRP_PHYS_PYB_GND, A, B, DEF, STG, CTL, HELP>, grid, blk, s, a, h); break;
        case ADRP_PHYS_PYB_DRAG: launch(hover_step_kernel<Real, ADRP_PHYS_PYB_DRAG, A, B, DEF, STG, CTL, HELP>, grid, blk, s, a, h); break;
        case ADRP_PHYS_PYB_DW: launch(hover_step_kernel<Real, ADRP_PHYS_PYB_DW, A, B, DEF, STG, CTL, HELP>, grid, blk, s, a, h); break;
        default: launch(hover_step_kernel<Real, ADRP_PHYS_PYB_GND_DRAG_DW, A, B, DEF, STG, CTL, HELP>, grid, blk, s, a, h); break;
    }
}

template <typename Real>
int hover_step(adrp_t* h, const float* act, float* obs, float* rew, uint8_t* term, uint8_t* trunc,
                      float* tobs, hipStream_t s) {
    HoverArgs<Real> a = hover_args<Real>(h);
    a.act = act; a.obs = obs; a.rew = rew; a.term = term; a.trunc = trunc; a.tobs = tobs;
    const dim3 grid((h->E + kBlock - 1) / kBlock);
    const int ph = h->cfg.physics;
    // compiled-in constants exist for the reference default (CF2X @ 240/30 Hz, B = 15)
    const bool stg = h->stage_rows && h->E % kBlock == 0;
    const bool help = h->cfg.autoreset && h->reset_helper;   // ADRP_RESET_HELPER=0 disables
    const int at = h->cfg.act_type;
    if (at == ADRP_ACT_PID || at == ADRP_ACT_VEL || at == ADRP_ACT_ONE_D_PID) {
        // fused DSLPIDControl: device-resident constants, runtime ring length
        if (at == ADRP_ACT_PID) launch_step_ph<Real, 3, 0, false, false, ADRP_ACT_PID>(a, ph, grid, s, h);
        else if (at == ADRP_ACT_VEL) launch_step_ph<Real, 4, 0, false, false, ADRP_ACT_VEL>(a, ph, grid, s, h);
        else launch_step_ph<Real, 1, 0, false, false, ADRP_ACT_ONE_D_PID>(a, ph, grid, s, h);
    } else if (h->cf2x && h->B == 15) {
        if (h->A == 1) launch_step_ph<Real, 1, 15, true>(a, ph, grid, s, h);
        else if (stg && help) launch_step_ph<Real, 4, 15, true, true, 0, true>(a, ph, grid, s, h);
        else if (stg) launch_step_ph<Real, 4, 15, true, true>(a, ph, grid, s, h);
        else launch_step_ph<Real, 4, 15, true>(a, ph, grid, s, h);
    } else if (h->A == 4 && h->B == 15 && stg) {
        if (help) launch_step_ph<Real, 4, 15, false, true, 0, true>(a, ph, grid, s, h);
        else launch_step_ph<Real, 4, 15, false, true>(a, ph, grid, s, h);
    } else if (h->A == 1) {
        if (h->B == 15) launch_step_ph<Real, 1, 15, false>(a, ph, grid, s, h);
        else launch_step_ph<Real, 1, 0, false>(a, ph, grid, s, h);
    } else {
        if (h->B == 15) launch_step_ph<Real, 4, 15, false>(a, ph, grid, s, h);
        else launch_step_ph<Real, 4, 0, false>(a, ph, grid, s, h);
    }
    HIPCHK(h, hipGetLastError());
    return ADRP_OK;
}

template <typename Real>
int hover_reset(adrp_t* h, const uint8_t* mask, float* obs, hipStream_t s) {
    HoverArgs<Real> a = hover_args<Real>(h);
    a.mask = mask; a.obs = obs;
    const dim3 grid((h->E + kBlock - 1) / kBlock);
    if (h->A == 1) hipLaunchKernelGGL((hover_reset_kernel<Real, 1>), grid, dim3(kBlock), 0, s, a);
    else if (h->A == 3) hipLaunchKernelGGL((hover_reset_kernel<Real, 3>), grid, dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL((hover_reset_kernel<Real, 4>), grid, dim3(kBlock), 0, s, a);
    HIPCHK(h, hipGetLastError());
    return ADRP_OK;
}
