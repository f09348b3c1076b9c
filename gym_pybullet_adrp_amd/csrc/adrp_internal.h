// adrp_internal.h — host-side handle and launch plumbing shared by the libadrp translation
// units (adrp.hip: the C-ABI; hover_f32/f64.hip, race_f32/f64.hip: kernel instantiations and
// their launchers, compiled in parallel).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <string.h>

#include <string>
#include <vector>

#include "../../include/adrp.h"
#include "hover_kernel.h"
#include "race_kernel.h"
#include "race_quad.h"
#include "device_guard.h"

using namespace adrp;

int seterr(adrp_t* h, int code, const std::string& msg);

struct adrp_handle {
    adrp_config cfg;
    int device = 0;
    int E = 0, N = 0, A = 0, D = 0, S = 0, B = 0;
    int nf_base = 0, ni = 0;
    size_t real_size = 4;
    void* f = nullptr;        // Real [nf_base][E*N]
    float* ring = nullptr;    // [B*A][E]
    int32_t* ist = nullptr;   // [ni][E*N]
    int32_t* counters = nullptr;  // device diagnostics (ground-model hits)
    void* cblk = nullptr;         // device HoverConst<Real> + HoverReset<Real>
    bool cf2x = false;            // compiled-in constants (hover_step_kernel<..., DEF=true>)
    bool stage_rows = true;       // LDS-staged obs rows when E % 64 == 0 (ADRP_STAGE_ROWS=0 disables)
    bool reset_helper = true;     // staged kernels: reset states from a helper wave (ADRP_RESET_HELPER=0)
    bool race_helpers = true;     // race fp32: helper waves (track copy, draws) (ADRP_RACE_HELPERS=0)
    bool race_quad = true;        // race: four lanes per drone (race_quad.h) (ADRP_RACE_QUAD=0: one lane)
    bool race_refine = true;      // race: support-function bounds before GJK (ADRP_RACE_REFINE=0: centre bounds only)
    bool race_cf2x = false;       // race: the physical constants are race_cf2x_phys' (the quad kernel's literals)
    bool race_predraw = true;     // race quad: sub-step draws up front into LDS (ADRP_RACE_PREDRAW=0: in the loop)
    float* cmdf = nullptr;        // race command mode (adrp_enable_commands): [ADRP_CMD_NF][E*N]
    int32_t* cmdi = nullptr;      // [ADRP_CMD_NI][E*N]
    const double* inj_act = nullptr;    // adrp_set_noise (parity mode): caller's device arrays
    const double* inj_force = nullptr;
    int diagnostics = 0;
    uint32_t* mom_hash = nullptr; // race diagnostics: [E*N] firmware int16-moment hash of the last step
    int16_t* mom_log = nullptr;   // race diagnostics level 2: [E*N][S][3] the last step's int16 moments
    int32_t* mom_log_n = nullptr; //   [E*N] firmware calls per drone
    // race next-reset images (race_quad.h race_refill_q4; four-lane kernel with auto-reset): refilled
    // by a launch every img_period steps (ADRP_RESET_IMAGES=K, 0 = off)
    void* img_f = nullptr;        // Real [RF_N][E*N]
    int32_t* img_i = nullptr;     // [RI_N][E*N]
    float* img_row = nullptr;     // [E*N][D]
    int32_t* img_ep = nullptr;    // [E], -1 = none
    int img_period = 32;
    unsigned img_ctr = 0;
    // persistent step (adrp_persistent_*, hover_persist.h): host-mapped mailbox and its own stream
    void* pbox = nullptr;         // host address of the mapped mailbox (PersistCtl + buffers), or null
    hipStream_t pstream = nullptr;
    uint32_t pseq = 0;
    bool pline = false;           // line mode: action + request tag in one 64-byte line (E * A <= 15)
    size_t poff[6] = {0, 0, 0, 0, 0, 0};   // act, obs, rew, term, trunc, tobs byte offsets in pbox
    // SB3 host path (adrp_vec_bind / adrp_vec_step): the bound slots, host pointers translated
    adrp_vec_io vio[ADRP_VEC_SLOTS];
    bool vbound[ADRP_VEC_SLOTS] = {false, false, false, false};
    // kernel timing (adrp_profile_begin/end)
    std::vector<hipEvent_t> ev_start, ev_stop;
    int prof_cap = 0, prof_n = 0;
    std::string err;
};



#define HIPCHK(h, x)                                                                            \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess)                                                                   \
            return seterr(h, ADRP_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_));  \
    } while (0)

constexpr int kBlock = kStepBlock;

inline int race_group(int n) { return n <= 1 ? 1 : n <= 2 ? 2 : n <= 4 ? 4 : 8; }

// the four-lane race kernel (race_quad.h) runs a handle when: it is not switched off
// (ADRP_RACE_QUAD=0); fp64 only for the reference drone (compiled-in constants, race_is_cf2x);
// disturbances, if on, drawn up front (S <= kRacePreS, ADRP_RACE_PREDRAW not 0); no parity-mode
// injection (adrp_set_noise).  Every other handle runs the one-lane kernel (race_kernel.h), which
// covers all of these with the same arithmetic (test_quad_matches_lane).
inline bool race_quad_ok(const adrp_t* h) {
    // (diagnostics level 2, the firmware moment log, is the one-lane kernel's)
    return h->race_quad && h->diagnostics < 2 && (h->race_cf2x || h->real_size == 4) && !h->inj_force &&
           !(h->cfg.track.disturbances && (h->S > kRacePreS || !h->race_predraw));
}

// HoverAviary action width (BaseRLAviary._actionSpace, BaseRLAviary.py:141-147) and whether the
// action type runs the fused DSLPIDControl
inline bool hover_has_pid(int t) { return t == ADRP_ACT_PID || t == ADRP_ACT_VEL || t == ADRP_ACT_ONE_D_PID; }
inline int hover_act_dim(int t) {
    return t == ADRP_ACT_PID ? 3 : (t == ADRP_ACT_ONE_D_RPM || t == ADRP_ACT_ONE_D_PID) ? 1 : 4;
}

template <typename Real>
inline HoverArgs<Real> hover_args(const adrp_t* h) {
    const adrp_config& c = h->cfg;
    HoverArgs<Real> a;
    memset(&a, 0, sizeof a);
    a.c = (const HoverConst<Real>*)h->cblk;
    a.r = (const HoverReset<Real>*)((const char*)h->cblk + sizeof(HoverConst<Real>));
    a.E = h->E; a.B = h->B; a.D = h->D;
    a.autoreset = c.autoreset;
    a.seed = c.seed;
    a.env_offset = c.env_offset;
    a.f = (Real*)h->f;
    a.ring = h->ring;
    a.ist = h->ist;
    a.contact_count = h->diagnostics ? h->counters : nullptr;
    return a;
}

template <typename Real>
constexpr size_t race_ticks_offset() { return (sizeof(RaceConst<Real>) + 255) & ~size_t(255); }

template <typename Real>
inline RaceArgs<Real> race_args(const adrp_t* h) {
    RaceArgs<Real> a;
    memset(&a, 0, sizeof a);
    a.c = (const RaceConst<Real>*)h->cblk;
    a.ticks = (const uint32_t*)((const char*)h->cblk + race_ticks_offset<Real>());
    a.f = (Real*)h->f;
    a.ist = h->ist;
    a.seed = h->cfg.seed;
    a.env_offset = h->cfg.env_offset;
    a.E = h->E;
    a.cf = h->cmdf;
    a.ci = h->cmdi;
    a.inj_act = h->inj_act;
    a.inj_force = h->inj_force;
    a.mom_hash = h->diagnostics ? h->mom_hash : nullptr;
    a.mom_log = h->diagnostics >= 2 ? h->mom_log : nullptr;
    a.mom_log_n = h->diagnostics >= 2 ? h->mom_log_n : nullptr;
    a.img_f = (Real*)h->img_f;
    a.img_i = h->img_i;
    a.img_row = h->img_row;
    a.img_ep = h->img_ep;
    a.reset_count = h->diagnostics ? h->counters + 1 : nullptr;
    return a;
}

// launchers (one translation unit per task x precision)
template <typename Real>
int hover_step(adrp_t* h, const float* act, float* obs, float* rew, uint8_t* term, uint8_t* trunc, float* tobs,
               hipStream_t s);
template <typename Real>
int hover_reset(adrp_t* h, const uint8_t* mask, float* obs, hipStream_t s);
template <typename Real>
int hover_persist_launch(adrp_t* h, const HoverArgs<Real>& a, void* ctl, hipStream_t s);
template <typename Real>
int race_step(adrp_t* h, const float* act, float* obs, float* rew, uint8_t* term, uint8_t* trunc, float* tobs,
              hipStream_t s);
template <typename Real>
int race_reset(adrp_t* h, const uint8_t* mask, float* obs, hipStream_t s);
template <typename Real>
int race_command(adrp_t* h, const int32_t* cmd, const double* args, hipStream_t s);
template <typename Real>
int race_cmd_init(adrp_t* h, hipStream_t s);

#ifdef ADRP_RACE_TIMING
// each kernel translation unit is its own code object with its own g_race_phase
int phase_read_hover_f32(unsigned long long* out, int reset);
int phase_read_hover_f64(unsigned long long* out, int reset);
int phase_read_race_f32(unsigned long long* out, int reset);
int phase_read_race_f64(unsigned long long* out, int reset);
int phase_read_race_f32b(unsigned long long* out, int reset);
int phase_read_race_f32c(unsigned long long* out, int reset);
int phase_read_race_f64b(unsigned long long* out, int reset);
int phase_read_race_f64c(unsigned long long* out, int reset);
int wave_read_race_f32(unsigned long long* out, int n);
int wave_read_race_f64(unsigned long long* out, int n);
#define ADRP_PHASE_READER(name)                                                                  \
    int name(unsigned long long* out, int reset) {                                               \
        if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_race_phase), 32 * sizeof(unsigned long long)) != hipSuccess) \
            return ADRP_ERR_DEVICE;                                                              \
        if (reset) {                                                                             \
            static const unsigned long long z[32] = {};                                          \
            if (hipMemcpyToSymbol(HIP_SYMBOL(g_race_phase), z, sizeof z) != hipSuccess) return ADRP_ERR_DEVICE; \
        }                                                                                        \
        return ADRP_OK;                                                                          \
    }
#ifdef ADRP_RACE_GJK_STATS
int gjk_dump_read_f32(double* out, int max, int reset);
int gjk_dump_read_f64(double* out, int max, int reset);
#define ADRP_GJK_DUMP_READER(name)                                                               \
    int name(double* out, int max, int reset) {                                                  \
        unsigned int n = 0;                                                                      \
        if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_gjk_dump_n), sizeof n) != hipSuccess) return -1; \
        const int m = int(n < unsigned(kGjkDumps) ? n : unsigned(kGjkDumps));                   \
        const int c = m < max ? m : max;                                                         \
        if (c > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gjk_dump), size_t(c) * kGjkDumpF * sizeof(double)) \
                         != hipSuccess) return -1;                                               \
        if (reset) { const unsigned int z = 0; if (hipMemcpyToSymbol(HIP_SYMBOL(g_gjk_dump_n), &z, sizeof z) != hipSuccess) return -1; } \
        return c;                                                                                \
    }
#endif
#define ADRP_WAVE_READER(name)                                                                   \
    int name(unsigned long long* out, int n) {                                                   \
        if (n < 0 || n > kWaveSlots) return ADRP_ERR_INVALID;                                    \
        return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_race_wave), size_t(n) * 8 * sizeof(unsigned long long)) \
                       == hipSuccess ? ADRP_OK : ADRP_ERR_DEVICE;                                 \
    }
#endif
