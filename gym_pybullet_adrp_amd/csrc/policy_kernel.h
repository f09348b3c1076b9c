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
// Layout: one block = 16 observation rows; all three layers run on the f32-input MFMA
// v_mfma_f32_16x16x4_f32 (exact f32 fma chains, no reduced precision), oriented so that each
// layer's accumulator tile is, element for element, the next layer's B operand:
//   H1ᵀ = W1 · Xᵀ,  H2ᵀ = W2 · act(H1ᵀ + b1),  Oᵀ = W3 · act(H2ᵀ + b2)
// A 16x16 f32 accumulator holds [unit = 16 t + 4 (lane >> 4) + reg][row = lane & 15]; as a
// B operand, k-step (t, reg) then covers units {16 t + 4 g + reg : g = 0..3}.  The host
// pre-permutes every weight tile into that k order ("fragments": 64 floats, one per lane),
// so the hand-off between layers is a same-lane LDS store / load with no transpose.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "adrp_device.h"

namespace adrp {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// fragment-blob layout (floats), written by the host (policy.hip: build_blob).  Layer 1 is
// always kPolicyS1 = 16 k-steps (in_dim <= 64, zero-padded weights), so no loop has a
// runtime trip count.
constexpr int kPolicyS1 = 16;
struct PolicyLayout {
    int in_dim;              // observation width (<= 4 * kPolicyS1)
    int f1, f2, f3;          // fragment offsets of layers 1..3 (in floats)
    int b1, b2, b3;          // bias offsets
    int total;               // blob size in floats
};

// action transform (RLController._action_transform variants)
enum { POLICY_RAW = 0, POLICY_RELATIVE = 1, POLICY_ABSOLUTE = 2 };

// tanh(x) = (e^2x - 1) / (e^2x + 1), branch-free on the hardware exp2 / rcp (|x| clamped to 15,
// where tanh is 1 in f32); absolute error ~1e-7, far inside the policy's 2e-5 bar.  OCML's
// tanhf branches per lane range, which splits the unrolled MFMA schedule into blocks.
__device__ __forceinline__ float tanh_fast(float x) {
    const float c = __builtin_amdgcn_fmed3f(x, -15.0f, 15.0f);
    const float t = __builtin_amdgcn_exp2f(c * 2.8853900817779268f);     // e^(2c)
    return (t - 1.0f) * __builtin_amdgcn_rcpf(t + 1.0f);
}

template <bool RELU>
__device__ __forceinline__ float policy_act(float x) {
    if constexpr (RELU) return x > 0.0f ? x : 0.0f;
    else return tanh_fast(x);
}

// map2pi(angle) = ((angle + pi) % (2 pi)) - pi with NumPy's floor-mod, in float64
__device__ __forceinline__ double map2pi_d(double a) {
    const double two_pi = 6.283185307179586, pi = 3.141592653589793;
    const double x = a + pi;
    double r = fmod(x, two_pi);
    if (r != 0.0 && r < 0.0) r += two_pi;
    return r - pi;
}

// T1 = H1 / 16, T2 = H2 / 16, RELU (else Tanh).  One block = 16 observation rows and
// NW = max(T1, T2) waves: wave w owns hidden-unit tile w of each layer, so a launch has
// NW x rows / 16 waves (all SIMDs busy at the race batch sizes) and each wave issues its few
// weight fragments (read straight from global memory: 256 contiguous bytes per fragment per
// wave, the blob L2-resident after the first waves) together with its observation loads, at
// entry: one memory latency per launch.  The activations between layers go through LDS in
// the B-operand order, so every read and write is conflict-free (lds[(tile*4 + reg)*64 + lane]).
// RT row tiles (16 rows each) per block reuse the weight fragments a wave holds in registers.
template <int T1, int T2, bool RELU, int RT>
__global__ void __launch_bounds__(512) policy_kernel(const float* __restrict__ blob, PolicyLayout L,
                                                     const float* __restrict__ obs, int rows, int obs_stride,
                                                     float* __restrict__ act, int mode) {
    __shared__ float h1s[T1 * 4 * 64];
    __shared__ float h2s[T2 * 4 * 64];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;          // wave = unit tile
    const int g = lane >> 4;
    const bool l1 = w < T1, l2 = w < T2;
    // ---- the weights this wave needs, issued up front, kept for all RT row tiles ----
    float w1f[kPolicyS1], w2f[T1][4], b1v[4], b2v[4];
#pragma unroll
    for (int s = 0; s < kPolicyS1; ++s) w1f[s] = blob[L.f1 + ((l1 ? w : 0) * kPolicyS1 + s) * 64 + lane];
#pragma unroll
    for (int t = 0; t < T1; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) w2f[t][i] = blob[L.f2 + (((l2 ? w : 0) * T1 + t) * 4 + i) * 64 + lane];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        b1v[i] = blob[L.b1 + 16 * (l1 ? w : 0) + 4 * g + i];
        b2v[i] = blob[L.b2 + 16 * (l2 ? w : 0) + 4 * g + i];
    }
    float w3f[T2][4], b3v[4];
    if (w == 0) {
#pragma unroll
        for (int u = 0; u < T2; ++u)
#pragma unroll
            for (int i = 0; i < 4; ++i) w3f[u][i] = blob[L.f3 + (u * 4 + i) * 64 + lane];
#pragma unroll
        for (int i = 0; i < 4; ++i) b3v[i] = blob[L.b3 + i];
    }
    for (int rt = 0; rt < RT; ++rt) {
    const int row0 = (blockIdx.x * RT + rt) * 16;
    if (row0 >= rows) return;                // block-uniform
    const int r = row0 + (lane & 15);
    const bool live = r < rows;
    const float* xrow = obs + size_t(live ? r : row0) * obs_stride;
    float xb[kPolicyS1];
#pragma unroll
    for (int s = 0; s < kPolicyS1; ++s) {
        const int k = 4 * s + g;
        const float v = xrow[k < L.in_dim ? k : 0];
        xb[s] = (live && k < L.in_dim) ? v : 0.0f;
    }

    // ---- layer 1, unit tile w: two interleaved accumulator chains over the 16 k-steps ----
    if (l1) {
        f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
#pragma unroll
        for (int s = 0; s < kPolicyS1; s += 2) {
            a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w1f[s], xb[s], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w1f[s + 1], xb[s + 1], a1, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) h1s[(w * 4 + i) * 64 + lane] = policy_act<RELU>(a0[i] + a1[i] + b1v[i]);
    }
    __syncthreads();
    // ---- layer 2, unit tile w: B operands = layer-1 tiles (t, reg) from LDS ----
    if (l2) {
        f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
#pragma unroll
        for (int t = 0; t < T1; ++t)
#pragma unroll
            for (int i = 0; i < 4; i += 2) {
                a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[t][i], h1s[(t * 4 + i) * 64 + lane], a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[t][i + 1], h1s[(t * 4 + i + 1) * 64 + lane], a1, 0, 0, 0);
            }
#pragma unroll
        for (int i = 0; i < 4; ++i) h2s[(w * 4 + i) * 64 + lane] = policy_act<RELU>(a0[i] + a1[i] + b2v[i]);
    }
    __syncthreads();
    if (w == 0) {
    // ---- layer 3 (action_net, 4 outputs padded to a 16-unit tile), wave 0 ----
    f32x4 o0 = f32x4{0.f, 0.f, 0.f, 0.f}, o1 = o0;
#pragma unroll
    for (int u = 0; u < T2; ++u)
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
            o0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w3f[u][i], h2s[(u * 4 + i) * 64 + lane], o0, 0, 0, 0);
            o1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w3f[u][i + 1], h2s[(u * 4 + i + 1) * 64 + lane], o1, 0, 0, 0);
        }
    // lanes 0..15 hold the 4 outputs of row (lane & 15)
    if (g == 0 && live) {
    float a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float m = o0[i] + o1[i] + b3v[i];
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
    }
    __syncthreads();          // h1s / h2s are rewritten by the next row tile
    }
}

// ---- PPO rollout step: actor + critic + diagonal-Gaussian sample ----------
// SB3 2.3.2 OnPolicyAlgorithm.collect_rollouts: actions, values, log_probs = policy(obs) with
// ActorCriticPolicy.forward(obs, deterministic=False): latent_pi / latent_vf = the two MLPs of
// mlp_extractor, mean = action_net(latent_pi), value = value_net(latent_vf),
// DiagGaussianDistribution(mean, exp(log_std)).sample() = mean + std * eps, log_prob = sum over the
// action dims of Normal.log_prob; the env then gets clip(action, low, high) (and here the
// RLController transform).  One block = 16 rows and 2 NW waves: waves [0, NW) run the actor's
// hidden layers, waves [NW, 2 NW) the critic's, on their own LDS tiles (same barrier sequence);
// wave 0 finishes the action, wave NW the value.  eps: one Philox4x32-10 block per row, counter
// {row, counter, kTagPolicy, 0}, Box-Muller by normal_pair_f (the oracle's restatement draws the
// same floats).
constexpr uint32_t kTagPolicy = 0x504f4c00u;   // "POL"

struct PolicySampleArgs {
    const float* actor;   PolicyLayout La;      // fragment blobs (build_blob) of the two MLPs
    const float* critic;  PolicyLayout Lc;
    const float* log_std;                       // [act_dim]
    const float* obs; int rows, obs_stride, mode, act_dim;
    uint64_t seed; uint32_t counter;
    float* env_act;     // [rows][act_dim == 4 ? 4 : act_dim] clip + transform
    float* action;      // [rows][act_dim] the sample (rollout-buffer action)
    float* value;       // [rows]
    float* log_prob;    // [rows]
    float* eps;         // [rows][act_dim] or null
};

// hidden layers of one MLP for the 16 rows of xb: unit tile w of layer 1 / 2 into h1s / h2s (two
// barriers, taken by every wave of the block)
template <int T1, int T2, bool RELU>
__device__ __forceinline__ void policy_hidden(const float* __restrict__ blob, const PolicyLayout& L, int w, int lane,
                                              const float (&xb)[kPolicyS1], float* h1s, float* h2s) {
    const int g = lane >> 4;
    const bool l1 = w < T1, l2 = w < T2;
    if (l1) {
        f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
#pragma unroll
        for (int s = 0; s < kPolicyS1; s += 2) {
            a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(blob[L.f1 + (w * kPolicyS1 + s) * 64 + lane], xb[s], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(blob[L.f1 + (w * kPolicyS1 + s + 1) * 64 + lane], xb[s + 1], a1, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
            h1s[(w * 4 + i) * 64 + lane] = policy_act<RELU>(a0[i] + a1[i] + blob[L.b1 + 16 * w + 4 * g + i]);
    }
    __syncthreads();
    if (l2) {
        f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
#pragma unroll
        for (int t = 0; t < T1; ++t)
#pragma unroll
            for (int i = 0; i < 4; i += 2) {
                a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(blob[L.f2 + ((w * T1 + t) * 4 + i) * 64 + lane],
                                                          h1s[(t * 4 + i) * 64 + lane], a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(blob[L.f2 + ((w * T1 + t) * 4 + i + 1) * 64 + lane],
                                                          h1s[(t * 4 + i + 1) * 64 + lane], a1, 0, 0, 0);
            }
#pragma unroll
        for (int i = 0; i < 4; ++i)
            h2s[(w * 4 + i) * 64 + lane] = policy_act<RELU>(a0[i] + a1[i] + blob[L.b2 + 16 * w + 4 * g + i]);
    }
    __syncthreads();
}

// the output layer (a 16-unit tile, outputs < n_out live) of the MLP whose layer-2 tiles are in h2s
template <int T2>
__device__ __forceinline__ f32x4 policy_out(const float* __restrict__ blob, const PolicyLayout& L, int lane,
                                            const float* h2s) {
    f32x4 o0 = f32x4{0.f, 0.f, 0.f, 0.f}, o1 = o0;
#pragma unroll
    for (int u = 0; u < T2; ++u)
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
            o0 = __builtin_amdgcn_mfma_f32_16x16x4f32(blob[L.f3 + (u * 4 + i) * 64 + lane], h2s[(u * 4 + i) * 64 + lane],
                                                      o0, 0, 0, 0);
            o1 = __builtin_amdgcn_mfma_f32_16x16x4f32(blob[L.f3 + (u * 4 + i + 1) * 64 + lane],
                                                      h2s[(u * 4 + i + 1) * 64 + lane], o1, 0, 0, 0);
        }
    return o0 + o1;
}

template <int T1, int T2, bool RELU>
__global__ void __launch_bounds__(1024) policy_sample_kernel(PolicySampleArgs a) {
    constexpr int NW = T1 > T2 ? T1 : T2;
    __shared__ float h1s[2][T1 * 4 * 64];
    __shared__ float h2s[2][T2 * 4 * 64];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int net = wave >= NW ? 1 : 0;            // 0 actor, 1 critic
    const int w = wave - net * NW;
    const int g = lane >> 4;
    const int row0 = blockIdx.x * 16;
    const int r = row0 + (lane & 15);
    const bool live = r < a.rows;
    const float* xrow = a.obs + size_t(live ? r : row0) * a.obs_stride;
    const PolicyLayout& L = net ? a.Lc : a.La;
    const float* blob = net ? a.critic : a.actor;
    float xb[kPolicyS1];
#pragma unroll
    for (int s = 0; s < kPolicyS1; ++s) {
        const int k = 4 * s + g;
        const float v = xrow[k < L.in_dim ? k : 0];
        xb[s] = (live && k < L.in_dim) ? v : 0.0f;
    }
    policy_hidden<T1, T2, RELU>(blob, L, w, lane, xb, h1s[net], h2s[net]);
    if (w != 0) return;                              // waves 0 / NW finish (wave-uniform exit)
    const f32x4 o = policy_out<T2>(blob, L, lane, h2s[net]);   // the MFMA needs all 64 lanes
    if (g != 0 || !live) return;                     // lanes 0..15: the outputs of row lane & 15
    if (net == 1) {                                  // value_net: output 0
        a.value[r] = o[0] + blob[L.b3];
        return;
    }
    // Philox block of this row -> 4 standard normals (act_dim <= 4 of them used)
    const U4 u = philox4x32_10(U4{uint32_t(r), a.counter, kTagPolicy, 0u}, uint32_t(a.seed), uint32_t(a.seed >> 32));
    float eps[4];
    normal_pair_f(u.a, u.b, &eps[0], &eps[1]);
    normal_pair_f(u.c, u.d, &eps[2], &eps[3]);
    float act[4], clipped[4], lp = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const bool on = i < a.act_dim;
        const float mean = o[i] + blob[L.b3 + i];
        const float ls = on ? a.log_std[i] : 0.0f;
        const float sd = expf(ls);
        const float x = mean + sd * eps[i];
        // torch Normal.log_prob: -((x - loc)^2) / (2 var) - log(scale) - log(sqrt(2 pi))
        const float d = x - mean;
        const float l = -(d * d) / (2.0f * sd * sd) - ls - 0.91893853320467274f;
        lp += on ? l : 0.0f;
        act[i] = x;
        clipped[i] = x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
        if (on) {
            a.action[size_t(r) * a.act_dim + i] = x;
            if (a.eps) a.eps[size_t(r) * a.act_dim + i] = eps[i];
        }
    }
    (void)act;
    a.log_prob[r] = lp;
    if (a.mode == POLICY_RAW) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (i < a.act_dim) a.env_act[size_t(r) * a.act_dim + i] = clipped[i];
    } else {   // RLController / RLControllerTwoGates transform of the clipped action (act_dim 4)
        const bool rel = a.mode == POLICY_RELATIVE;
        const double px = rel ? double(xrow[0]) : 0.0, py = rel ? double(xrow[1]) : 0.0,
                     pz = rel ? double(xrow[2]) : 0.0, pyaw = rel ? double(xrow[5]) : 0.0;
        reinterpret_cast<float4*>(a.env_act)[r] =
            make_float4(float(px + double(clipped[0])), float(py + double(clipped[1])), float(pz + double(clipped[2])),
                        float(map2pi_d(pyaw + 0.0 * 3.141592653589793)));
    }
}

}  // namespace adrp
