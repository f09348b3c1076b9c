// policy_kernel.h — fused on-device actor forward of an SB3 PPO MlpPolicy (two hidden layers)
// plus the RLController action transform, for closed-loop MultiRaceAviary rollouts with no
// host round-trip.
//
// Reference path (FelixWaiblinger/gym-pybullet-adrp @ 2024-10-08):
//   RLController.predict / _action_transform      user_controller/RLController.py:39-73
//   RLControllerTwoGates._action_transform        user_controller/RLControllerTwoGates.py:56-69
//   PPO.predict(obs, deterministic=True)          stable_baselines3 2.3.2 (the zips' version):
//     ActorCriticPolicy: Flatten -> mlp_extractor.policy_net (Linear, act, Linear, act)
//     -> action_net (Linear) = the Gaussian mean; BasePolicy.predict clips it to the Box [-1, 1]
//   map2pi                                        gym_pybullet_adrp/utils/utils.py:188-197
//
// Layout: one wave = 16 observation rows; all three layers run on the f32-input MFMA
// v_mfma_f32_16x16x4_f32 (exact f32 fma chains, no reduced precision), oriented so that each
// layer's accumulator tile is the next layer's B operand with no lane movement:
//   H1ᵀ = W1 · Xᵀ,  H2ᵀ = W2 · act(H1ᵀ + b1),  Oᵀ = W3 · act(H2ᵀ + b2)
// A 16x16 f32 accumulator holds [unit = 16 t + 4 (lane >> 4) + reg][row = lane & 15]; as a
// B operand, k-step (t, reg) then covers units {16 t + 4 g + reg : g = 0..3}.  The host
// pre-permutes every weight tile into that k order ("fragments": 64 floats, one per lane,
// read conflict-free from LDS), so no layer needs a transpose or an LDS round trip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace adrp {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// fragment-blob layout (floats), written by the host (policy.hip: build_blob)
struct PolicyLayout {
    int in_dim, s1;          // observation width, k-steps of layer 1 (ceil(in_dim / 4))
    int f1, f2, f3;          // fragment offsets of layers 1..3 (in floats)
    int b1, b2, b3;          // bias offsets
    int total;               // blob size in floats
};

// action transform (RLController._action_transform variants)
enum { POLICY_RAW = 0, POLICY_RELATIVE = 1, POLICY_ABSOLUTE = 2 };

__device__ __forceinline__ float policy_act(float x, int relu) {
    return relu ? (x > 0.0f ? x : 0.0f) : tanhf(x);
}

// map2pi(angle) = ((angle + pi) % (2 pi)) - pi with NumPy's floor-mod, in float64
__device__ __forceinline__ double map2pi_d(double a) {
    const double two_pi = 6.283185307179586, pi = 3.141592653589793;
    const double x = a + pi;
    double r = fmod(x, two_pi);
    if (r != 0.0 && r < 0.0) r += two_pi;
    return r - pi;
}

// T1 = H1 / 16, T2 = H2 / 16.  Block = 4 waves = 64 rows; the blob is staged in LDS once.
template <int T1, int T2>
__global__ void __launch_bounds__(256) policy_kernel(const float* __restrict__ blob, PolicyLayout L,
                                                     const float* __restrict__ obs, int rows, int obs_stride,
                                                     float* __restrict__ act, int mode, int relu) {
    extern __shared__ float lds[];
    {   // stage the fragment blob (float4, whole block)
        const float4* src = reinterpret_cast<const float4*>(blob);
        float4* dst = reinterpret_cast<float4*>(lds);
        const int n4 = L.total >> 2;
        for (int k = threadIdx.x; k < n4; k += blockDim.x) dst[k] = src[k];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
    if (row0 >= rows) return;                      // whole wave out of range (after the barrier)
    const int r = row0 + (lane & 15);
    const bool live = r < rows;
    const int g = lane >> 4;
    const float* xrow = obs + size_t(live ? r : row0) * obs_stride;

    // ---- layer 1: H1ᵀ[16 t + ...][row] = Σ_k W1[unit][k] X[row][k] ----
    f32x4 h1[T1];
#pragma unroll
    for (int t = 0; t < T1; ++t) h1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < L.s1; ++s) {
        const int k = 4 * s + g;
        const float xb = (live && k < L.in_dim) ? xrow[k] : 0.0f;
#pragma unroll
        for (int t = 0; t < T1; ++t) {
            const float wa = lds[L.f1 + (t * L.s1 + s) * 64 + lane];
            h1[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa, xb, h1[t], 0, 0, 0);
        }
    }
#pragma unroll
    for (int t = 0; t < T1; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) h1[t][i] = policy_act(h1[t][i] + lds[L.b1 + 16 * t + 4 * g + i], relu);

    // ---- layer 2: the layer-1 accumulators are the B operands ----
    f32x4 h2[T2];
#pragma unroll
    for (int u = 0; u < T2; ++u) h2[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < T1; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int u = 0; u < T2; ++u) {
                const float wa = lds[L.f2 + ((u * T1 + t) * 4 + i) * 64 + lane];
                h2[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa, h1[t][i], h2[u], 0, 0, 0);
            }
#pragma unroll
    for (int u = 0; u < T2; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) h2[u][i] = policy_act(h2[u][i] + lds[L.b2 + 16 * u + 4 * g + i], relu);

    // ---- layer 3 (action_net, 4 outputs padded to a 16-unit tile) ----
    f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < T2; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float wa = lds[L.f3 + (u * 4 + i) * 64 + lane];
            o = __builtin_amdgcn_mfma_f32_16x16x4f32(wa, h2[u][i], o, 0, 0, 0);
        }
    // lanes 0..15 hold the 4 outputs of row (lane & 15) in o[0..3]
    if (g != 0 || !live) return;
    float a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float m = o[i] + lds[L.b3 + i];
        a[i] = m < -1.0f ? -1.0f : (m > 1.0f ? 1.0f : m);     // np.clip(actions, low, high)
    }
    float4 out;
    if (mode == POLICY_RAW) {
        out = make_float4(a[0], a[1], a[2], a[3]);
    } else {
        // action[3] = 0; target = pose + a * [1, 1, 1, pi] (RELATIVE, pose = obs[[0,1,2,5]]) or
        // a * [1, 1, 1, pi] (ABSOLUTE); yaw = map2pi(.) -- float32 action x float64 scale
        const bool rel = mode == POLICY_RELATIVE;
        const double px = rel ? double(xrow[0]) : 0.0, py = rel ? double(xrow[1]) : 0.0,
                     pz = rel ? double(xrow[2]) : 0.0, pyaw = rel ? double(xrow[5]) : 0.0;
        out = make_float4(float(px + double(a[0])), float(py + double(a[1])), float(pz + double(a[2])),
                          float(map2pi_d(pyaw + 0.0 * 3.141592653589793)));
    }
    reinterpret_cast<float4*>(act)[r] = out;
}

}  // namespace adrp
