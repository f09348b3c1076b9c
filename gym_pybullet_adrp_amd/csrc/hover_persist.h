// hover_persist.h — persistent HoverAviary step for small E (BASELINE config 1: one env stepped
// synchronously from Python, examples/pid.py:101-147 driving envs/BaseAviary.py:262-387).
//
// A launch per env.step costs the host a kernel launch (~5 us), the kernel a cold start (the
// agent-scope acquire at kernel start invalidates L2, so the first loads go to HBM) and the host a
// completion wait.  Here ONE launch stays resident on one CU per 64 envs and polls a host-mapped
// mailbox: the host writes the action into mapped memory and bumps `req`; the kernel runs the same
// hover_step_body as hover_step_kernel (the env state stays hot in L2 between steps), writes obs /
// reward / flags straight into mapped memory and publishes `done`.  The host spins on `done` in its
// own memory, so one env.step is two PCIe crossings and the step itself.
//
// Exit: the host's stop request, or no request for kPersistIdleTicks (s_memrealtime, 100 MHz).  The
// idle exit is ONE grid-wide decision: only workgroup 0 times out; it publishes `kstop` before it
// leaves and the other workgroups leave when they see it.  Every workgroup marks `exited[b]` on
// its way out, so a host that posted a request just as workgroup 0 timed out fails fast (the
// step may be partial) instead of waiting on a done word that never comes.  Every wave reaches
// one of the exits, so the grid always drains (a host that died leaves a kernel that ends by
// itself).
#pragma once

#include "hover_kernel.h"

namespace adrp {

constexpr uint32_t kPersistStop = 0xFFFFFFFFu;
constexpr int kPersistMaxBlocks = 16;                     // E <= 16 * 64 envs
constexpr uint64_t kPersistIdleTicks = 1000000000ull;     // 10 s without a request ends the kernel
constexpr int kPersistLineWords = 16;                     // line mode: 64-byte action line, tag in word 15

// the control block at the head of the mapped mailbox
struct PersistCtl {
    uint32_t req;                        // host: sequence number of the requested step, kPersistStop
    uint32_t status;                     // device: 1 running, 2 exited
    uint32_t kstop;                      // device (workgroup 0): idle timeout, every workgroup leaves
    uint32_t pad[13];
    uint32_t done[kPersistMaxBlocks];    // device: per workgroup, the last request it finished
    uint32_t exited[kPersistMaxBlocks];  // device: per workgroup, 1 once it has left the loop
};

// a: HoverArgs whose act / obs / rew / term / trunc / tobs point into the mapped mailbox (device
// addresses of host memory); f / ring / ist / c / r are the handle's device buffers.
// Memory traffic with the host, per step and without a cache-wide fence (a system-scope acquire
// would invalidate the L2 the env state lives in, a system-scope release would write it back):
//   - the request word and the action rows are read with system-scope atomic loads (no GPU cache
//     serves them); the action loads are issued after the load that saw req, and the host stored
//     the action before it published req;
//   - the outputs are plain stores into the same mapping; every wave waits for their completion,
//     then one lane per block runs a system-scope release (an L2 write-back: the env state lines
//     become clean, they are not evicted) and stores done; the host reads the outputs after it
//     sees done.  Without the release the done word could reach host memory before the last
//     output rows (seen once in the E = 70 bit-identity test: 69 stale obs words at step 1).
//
// LINE (E * A <= 15, one workgroup: BASELINE config 1's single env): the action floats and the
// request tag share ONE 64-byte line of the mailbox (tag in its last word, written by the host after
// the floats).  The wave polls the whole line with one 16-lane load, so the load that sees the new
// tag has already brought the action: one host round trip per step instead of two (tag, then rows).
template <typename Real, int PH, int A, int B, bool DEF, bool LINE>
__global__ void __launch_bounds__(kStepBlock) hover_persist_kernel(HoverArgs<Real> a, PersistCtl* ctl) {
    __shared__ uint32_t cmd;
    if (blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(&ctl->status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t last = 0;
    uint64_t t_idle = __builtin_amdgcn_s_memrealtime();
    if constexpr (LINE) {
        static_assert(kStepBlock == 64, "line mode: one wave per workgroup");
        const uint32_t* line = reinterpret_cast<const uint32_t*>(a.act);
        const int lane = threadIdx.x;
        for (;;) {
            uint32_t v = 0, r;
            for (;;) {
                if (lane < kPersistLineWords)
                    v = __hip_atomic_load(line + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                r = __builtin_amdgcn_readlane(v, kPersistLineWords - 1);
                if (r != last) break;
                if (__builtin_amdgcn_s_memrealtime() - t_idle > kPersistIdleTicks) {
                    r = kPersistStop;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (r == kPersistStop) break;
            float pre[A];
            const int src = (lane < a.E ? lane : a.E - 1) * A;   // lanes >= E: env E - 1's (E = 1: every lane runs env 0)
#pragma unroll
            for (int j = 0; j < A; ++j) pre[j] = __uint_as_float(__shfl(v, src + j));
            if constexpr (DEF) {
                constexpr HoverConst<Real> C = cf2x_consts<Real>(PH);
                hover_step_body<Real, PH, A, B, C.S, false, 0, false, 2>(a, C, pre);
            } else {
                hover_step_body<Real, PH, A, B, 0, false, 0, false, 2>(a, *a.c, pre);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(&ctl->done[0], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            last = r;
            t_idle = __builtin_amdgcn_s_memrealtime();
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (lane == 0) {
            __hip_atomic_store(&ctl->exited[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&ctl->status, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
    }
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t r;
            for (;;) {
                r = __hip_atomic_load(&ctl->req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (r != last) break;
                if (blockIdx.x == 0) {
                    if (__builtin_amdgcn_s_memrealtime() - t_idle > kPersistIdleTicks) {
                        __hip_atomic_store(&ctl->kstop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        r = kPersistStop;
                        break;
                    }
                } else if (__hip_atomic_load(&ctl->kstop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
                    r = kPersistStop;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            cmd = r;
        }
        __syncthreads();
        const uint32_t r = cmd;
        __syncthreads();   // cmd is rewritten by the next poll
        if (r == kPersistStop) break;
        if constexpr (DEF) {
            constexpr HoverConst<Real> C = cf2x_consts<Real>(PH);
            hover_step_body<Real, PH, A, B, C.S, false, 0, false, 1>(a, C);
        } else {
            hover_step_body<Real, PH, A, B, 0, false, 0, false, 1>(a, *a.c);
        }
        // every output store of every wave has completed, then ONE system-scope release makes them
        // visible to the host before done: a completed store is not yet a visible one (the flag can
        // overtake plain stores on their way to host memory).  The inline waits are invisible to
        // the compiler, which otherwise drops the wait after the release's write-back.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&ctl->done[blockIdx.x], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        last = r;
        t_idle = __builtin_amdgcn_s_memrealtime();
    }
    // the env state the next launch / get_state reads (kernel end releases it too)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(&ctl->exited[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(&ctl->status, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace adrp
