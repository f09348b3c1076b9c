// race_launch.h — MultiRaceAviary step/reset launchers (instantiated by race_f32.hip / race_f64.hip)
#pragma once

#include "adrp_internal.h"

// the quad kernel's physical constants are compiled in (race_cf2x_phys) for fp64, where that took
// config 4 from 98.2 to 95.5 us; for fp32 it measured 0.5 us slower (round-3 A/B)
template <typename Real>
constexpr bool kQuadDef = sizeof(Real) == 8;

// four lanes per drone (race_quad.h): 16 drones per 64-lane block
template <typename Real, int PH>
static void launch_race_q4(const RaceArgs<Real>& a, int G, hipStream_t s, adrp_t* h) {
    const bool draws = h->cfg.track.disturbances;   // (race_quad_ok: then drawn up front)
    const dim3 blk(kRaceBlock), grid((unsigned)((size_t(h->E) * G * 4 + kRaceBlock - 1) / kRaceBlock));
    auto go = [&](auto kernel) {
        if (h->prof_n < h->prof_cap) {
            hipExtLaunchKernelGGL(kernel, grid, blk, 0, s, h->ev_start[h->prof_n], h->ev_stop[h->prof_n], 0, a);
            ++h->prof_n;
        } else {
            hipLaunchKernelGGL(kernel, grid, blk, 0, s, a);
        }
    };
    auto by_g = [&](auto dr) {
        constexpr bool D = decltype(dr)::value;
        switch (G) {
#ifndef ADRP_DEV_FAST
            case 1: go(race_step_q4<Real, PH, 1, D, kQuadDef<Real>>); break;
            case 8: go(race_step_q4<Real, PH, 8, D, kQuadDef<Real>>); break;
#endif
            case 2: go(race_step_q4<Real, PH, 2, D, kQuadDef<Real>>); break;
            default: go(race_step_q4<Real, PH, 4, D, kQuadDef<Real>>); break;
        }
    };
    if (draws) by_g(std::true_type{});
    else by_g(std::false_type{});
}

// command mode: the lane kernel with the commander (commander.h), G = 8 lanes per env for every N
// (one instantiation per physics mode and precision; the commander path is for scripted
// controllers, not the benched RL step)
template <typename Real, int PH>
static void launch_race_cmd(const RaceArgs<Real>& a, hipStream_t s, adrp_t* h) {
    const dim3 blk(kRaceBlock), grid((unsigned)((size_t(h->E) * 8 + kRaceBlock - 1) / kRaceBlock));
    auto kernel = race_step_kernel<Real, PH, 8, 0, true>;
    if (h->prof_n < h->prof_cap) {
        hipExtLaunchKernelGGL(kernel, grid, blk, 0, s, h->ev_start[h->prof_n], h->ev_stop[h->prof_n], 0, a);
        ++h->prof_n;
    } else {
        hipLaunchKernelGGL(kernel, grid, blk, 0, s, a);
    }
}

template <typename Real, int PH>
static void launch_race_g(const RaceArgs<Real>& a, int G, hipStream_t s, adrp_t* h) {
    if (h->cmdf) return launch_race_cmd<Real, PH>(a, s, h);
    // the fp64 four-lane kernel has the reference drone's physical constants compiled in: another
    // drone (or PYB_FREQ) runs the one-lane kernel there
    if (race_quad_ok(h)) return launch_race_q4<Real, PH>(a, G, s, h);
    // kRaceBlock drone lanes, + kRaceHelpers helper waves per block in the fp32 kernel (the track
    // copy into LDS, and the sub-step draws with disturbances on; race_kernel.h)
    const int helpers = sizeof(Real) != 4 || !h->race_helpers ? 0
                        : h->cfg.track.disturbances && h->S <= kRacePreS ? 2 : 1;
    const dim3 blk(kRaceBlock * (helpers ? 1 + kRaceHelpers : 1)),
        grid((unsigned)((size_t(h->E) * G + kRaceBlock - 1) / kRaceBlock));
    auto go = [&](auto kernel) {
        if (h->prof_n < h->prof_cap) {
            hipExtLaunchKernelGGL(kernel, grid, blk, 0, s, h->ev_start[h->prof_n], h->ev_stop[h->prof_n], 0, a);
            ++h->prof_n;
        } else {
            hipLaunchKernelGGL(kernel, grid, blk, 0, s, a);
        }
    };
    constexpr bool F32 = sizeof(Real) == 4;
    auto by_g = [&](auto pre) {
        constexpr int P = decltype(pre)::value;
        switch (G) {
#ifndef ADRP_DEV_FAST
            case 1: go(race_step_kernel<Real, PH, 1, P>); break;
            case 8: go(race_step_kernel<Real, PH, 8, P>); break;
#endif
            case 2: go(race_step_kernel<Real, PH, 2, P>); break;
            default: go(race_step_kernel<Real, PH, 4, P>); break;
        }
    };
    if (helpers == 2) by_g(std::integral_constant<int, F32 ? 2 : 0>{});
    else if (helpers == 1) by_g(std::integral_constant<int, F32 ? 1 : 0>{});
    else by_g(std::integral_constant<int, 0>{});
}

// one physics mode's step kernels; explicitly instantiated in race_f32*.hip / race_f64*.hip so the
// physics modes compile in parallel translation units (the dispatching unit declares the others
// extern)
template <typename Real, int PH>
int race_step_ph(adrp_t* h, const RaceArgs<Real>& a, int G, hipStream_t s) {
    launch_race_g<Real, PH>(a, G, s, h);
    return ADRP_OK;
}
#define ADRP_RACE_STEP_PH(R, PH) int race_step_ph<R, PH>(adrp_t*, const RaceArgs<R>&, int, hipStream_t)

// the next-reset image refill (race_quad.h), in the step's lane layout
template <typename Real>
static void launch_race_refill(const RaceArgs<Real>& a, int G, hipStream_t s, adrp_t* h) {
    const dim3 blk(kRaceBlock), grid((unsigned)((size_t(h->E) * G * 4 + kRaceBlock - 1) / kRaceBlock));
    switch (G) {
#ifndef ADRP_DEV_FAST
        case 1: hipLaunchKernelGGL((race_refill_q4<Real, 1>), grid, blk, 0, s, a); break;
        case 8: hipLaunchKernelGGL((race_refill_q4<Real, 8>), grid, blk, 0, s, a); break;
#endif
        case 2: hipLaunchKernelGGL((race_refill_q4<Real, 2>), grid, blk, 0, s, a); break;
        default: hipLaunchKernelGGL((race_refill_q4<Real, 4>), grid, blk, 0, s, a); break;
    }
}

template <typename Real>
int race_step(adrp_t* h, const float* act, float* obs, float* rew, uint8_t* term, uint8_t* trunc,
                     float* tobs, hipStream_t s) {
    RaceArgs<Real> a = race_args<Real>(h);
    a.act = act; a.obs = obs; a.rew = rew; a.term = term; a.trunc = trunc; a.tobs = tobs;
    const int G = race_group(h->N);
    // next-reset images: the four-lane kernel's auto-reset copies them; refilled every img_period steps
    if (h->img_ep && !h->cmdf && race_quad_ok(h)) {
        if (h->img_ctr++ % unsigned(h->img_period) == 0) launch_race_refill<Real>(a, G, s, h);
    } else {
        a.img_f = nullptr; a.img_i = nullptr; a.img_row = nullptr; a.img_ep = nullptr;
    }
#ifdef ADRP_DEV_FAST   // experiment build (make dev): the benched race instantiations only
    if ((h->cfg.physics != ADRP_PHYS_PYB && h->cfg.physics != ADRP_PHYS_PYB_DW) || (G != 2 && G != 4))
        return seterr(h, ADRP_ERR_INVALID, "dev build: race config not instantiated");
    if (h->cfg.physics == ADRP_PHYS_PYB) race_step_ph<Real, ADRP_PHYS_PYB>(h, a, G, s);
    else race_step_ph<Real, ADRP_PHYS_PYB_DW>(h, a, G, s);
#else
    switch (h->cfg.physics) {
        case ADRP_PHYS_PYB: race_step_ph<Real, ADRP_PHYS_PYB>(h, a, G, s); break;
        case ADRP_PHYS_DYN: race_step_ph<Real, ADRP_PHYS_DYN>(h, a, G, s); break;
        case ADRP_PHYS_PYB_GND: race_step_ph<Real, ADRP_PHYS_PYB_GND>(h, a, G, s); break;
        case ADRP_PHYS_PYB_DRAG: race_step_ph<Real, ADRP_PHYS_PYB_DRAG>(h, a, G, s); break;
        case ADRP_PHYS_PYB_DW: race_step_ph<Real, ADRP_PHYS_PYB_DW>(h, a, G, s); break;
        default: race_step_ph<Real, ADRP_PHYS_PYB_GND_DRAG_DW>(h, a, G, s); break;
    }
#endif
    HIPCHK(h, hipGetLastError());
    return ADRP_OK;
}

template <typename Real>
int race_reset(adrp_t* h, const uint8_t* mask, float* obs, hipStream_t s) {
    RaceArgs<Real> a = race_args<Real>(h);
    a.mask = mask; a.obs = obs;
    const dim3 grid((unsigned)((size_t(h->E) * h->N + kRaceBlock - 1) / kRaceBlock));
    hipLaunchKernelGGL((race_reset_kernel<Real>), grid, dim3(kRaceBlock), 0, s, a);
    HIPCHK(h, hipGetLastError());
    return ADRP_OK;
}

template <typename Real>
int race_command(adrp_t* h, const int32_t* cmd, const double* args, hipStream_t s) {
    RaceArgs<Real> a = race_args<Real>(h);
    a.cmd = cmd; a.cargs = args;
    const dim3 grid((unsigned)((size_t(h->E) * h->N + kRaceBlock - 1) / kRaceBlock));
    hipLaunchKernelGGL((race_command_kernel<Real>), grid, dim3(kRaceBlock), 0, s, a);
    HIPCHK(h, hipGetLastError());
    return ADRP_OK;
}

template <typename Real>
int race_cmd_init(adrp_t* h, hipStream_t s) {
    RaceArgs<Real> a = race_args<Real>(h);
    const dim3 grid((unsigned)((size_t(h->E) * h->N + kRaceBlock - 1) / kRaceBlock));
    hipLaunchKernelGGL((race_cmd_init_kernel<Real>), grid, dim3(kRaceBlock), 0, s, a);
    HIPCHK(h, hipGetLastError());
    return ADRP_OK;
}
