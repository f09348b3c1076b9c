// policy.hip — C-ABI of the on-device policy forward (include/adrp.h: adrp_policy_*).
//
// Replaces, for the GPU batch, the per-drone RLController.predict -> PPO.predict chain
// (user_controller/RLController.py:39-73, RLControllerTwoGates.py:38-69): observation rows of
// adrp_step's obs buffer in, FULLSTATE setpoints for the next adrp_step out, on the same stream.
#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/adrp.h"
#include "policy_kernel.h"
#include "device_guard.h"

using namespace adrp;

int seterr(adrp_t* h, int code, const std::string& msg);

struct adrp_policy {
    int device = 0;
    int in_dim = 0, h1 = 0, h2 = 0, relu = 0, act_dim = 4;
    int row_tiles = 0;       // 16-row tiles per block (ADRP_POLICY_RT; 0 = default)
    PolicyLayout L{};
    float* blob = nullptr;   // device fragment blob
    PolicyLayout Lc{};       // critic (adrp_policy_set_critic)
    float* critic = nullptr;
    float* log_std = nullptr;
};

// Pre-permute the Linear weights (torch layout [out][in], row-major) into the per-lane MFMA
// fragments policy_kernel reads (see policy_kernel.h for the k order).
static std::vector<float> build_blob(int in_dim, int H1, int H2, const float* w1, const float* b1, const float* w2,
                                     const float* b2, const float* w3, const float* b3, PolicyLayout* L, int n_out = 4) {
    const int T1 = H1 / 16, T2 = H2 / 16, S1 = kPolicyS1;
    L->in_dim = in_dim;
    L->f1 = 0;
    L->f2 = L->f1 + T1 * S1 * 64;
    L->f3 = L->f2 + T2 * T1 * 4 * 64;
    L->b1 = L->f3 + T2 * 4 * 64;
    L->b2 = L->b1 + H1;
    L->b3 = L->b2 + H2;
    L->total = (L->b3 + 16 + 3) & ~3;
    std::vector<float> v(L->total, 0.0f);
    for (int t = 0; t < T1; ++t)
        for (int s = 0; s < S1; ++s)
            for (int l = 0; l < 64; ++l) {
                const int unit = 16 * t + (l & 15), k = 4 * s + (l >> 4);
                v[L->f1 + (t * S1 + s) * 64 + l] = k < in_dim ? w1[size_t(unit) * in_dim + k] : 0.0f;
            }
    for (int u = 0; u < T2; ++u)
        for (int t = 0; t < T1; ++t)
            for (int i = 0; i < 4; ++i)
                for (int l = 0; l < 64; ++l) {
                    const int out = 16 * u + (l & 15), k = 16 * t + 4 * (l >> 4) + i;
                    v[L->f2 + ((u * T1 + t) * 4 + i) * 64 + l] = w2[size_t(out) * H1 + k];
                }
    for (int u = 0; u < T2; ++u)
        for (int i = 0; i < 4; ++i)
            for (int l = 0; l < 64; ++l) {
                const int out = l & 15, k = 16 * u + 4 * (l >> 4) + i;
                v[L->f3 + (u * 4 + i) * 64 + l] = out < n_out ? w3[size_t(out) * H2 + k] : 0.0f;
            }
    memcpy(&v[L->b1], b1, sizeof(float) * H1);
    memcpy(&v[L->b2], b2, sizeof(float) * H2);
    memcpy(&v[L->b3], b3, sizeof(float) * n_out);
    return v;
}

template <int T1, int T2>
static hipError_t launch_policy(const adrp_policy_t* p, const float* obs, int rows, int stride, float* act, int mode,
                                hipStream_t s) {
    // row tiles per block: each block reuses its weight fragments over RT x 16 rows
    const int tiles = (rows + 15) / 16;
    int rt = p->row_tiles;
    if (rt == 0) rt = T1 >= 8 ? 2 : 1;   // measured (rocprof, MI355X): 49-64-64 @ 4096 rows best at 1,
                                          // 49-128-128 @ 16384 rows at 2 (tools/policy_probe.py)
    const dim3 grid((tiles + rt - 1) / rt), blk(64 * (T1 > T2 ? T1 : T2));
#define ADRP_POLICY_LAUNCH(R)                                                                                   \
    do {                                                                                                        \
        if (p->relu)                                                                                            \
            hipLaunchKernelGGL((policy_kernel<T1, T2, true, R>), grid, blk, 0, s, p->blob, p->L, obs, rows, stride, act, \
                               mode);                                                                           \
        else                                                                                                    \
            hipLaunchKernelGGL((policy_kernel<T1, T2, false, R>), grid, blk, 0, s, p->blob, p->L, obs, rows, stride,     \
                               act, mode);                                                                      \
    } while (0)
    if (rt >= 4) ADRP_POLICY_LAUNCH(4);
    else if (rt == 2) ADRP_POLICY_LAUNCH(2);
    else ADRP_POLICY_LAUNCH(1);
#undef ADRP_POLICY_LAUNCH
    return hipGetLastError();
}

template <int T1>
static hipError_t dispatch_t2(const adrp_policy_t* p, const float* obs, int rows, int stride, float* act, int mode,
                              hipStream_t s) {
    switch (p->h2 / 16) {
        case 1: return launch_policy<T1, 1>(p, obs, rows, stride, act, mode, s);
        case 2: return launch_policy<T1, 2>(p, obs, rows, stride, act, mode, s);
        case 4: return launch_policy<T1, 4>(p, obs, rows, stride, act, mode, s);
        default: return launch_policy<T1, 8>(p, obs, rows, stride, act, mode, s);
    }
}

static bool pow2_tiles(int h) { return h == 16 || h == 32 || h == 64 || h == 128; }

extern "C" int adrp_policy_create(int device, int in_dim, int hidden1, int hidden2, int activation, const float* w1,
                                  const float* b1, const float* w2, const float* b2, const float* w3, const float* b3,
                                  adrp_policy_t** out) {
    return adrp_policy_create2(device, in_dim, hidden1, hidden2, 4, activation, w1, b1, w2, b2, w3, b3, out);
}

static int upload(const std::vector<float>& v, float** dst) {
    if (hipMalloc((void**)dst, v.size() * sizeof(float)) != hipSuccess) return ADRP_ERR_OOM;
    if (hipMemcpy(*dst, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
        hipFree(*dst);
        *dst = nullptr;
        return ADRP_ERR_DEVICE;
    }
    return ADRP_OK;
}

extern "C" int adrp_policy_create2(int device, int in_dim, int hidden1, int hidden2, int act_dim, int activation,
                                   const float* w1, const float* b1, const float* w2, const float* b2, const float* w3,
                                   const float* b3, adrp_policy_t** out) {
    if (!out) return seterr(nullptr, ADRP_ERR_INVALID, "out is NULL");
    if (act_dim < 1 || act_dim > 4) return seterr(nullptr, ADRP_ERR_INVALID, "policy act_dim must be 1..4");
    *out = nullptr;
    if (!w1 || !b1 || !w2 || !b2 || !w3 || !b3) return seterr(nullptr, ADRP_ERR_INVALID, "NULL weight pointer");
    if (in_dim < 1 || in_dim > 4 * kPolicyS1) return seterr(nullptr, ADRP_ERR_INVALID, "policy in_dim must be 1..64");
    if (!pow2_tiles(hidden1) || !pow2_tiles(hidden2))
        return seterr(nullptr, ADRP_ERR_INVALID, "policy hidden sizes must be 16, 32, 64 or 128");
    if (activation != ADRP_POLICY_TANH && activation != ADRP_POLICY_RELU)
        return seterr(nullptr, ADRP_ERR_INVALID, "policy activation must be TANH or RELU");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return seterr(nullptr, ADRP_ERR_DEVICE, "no HIP device visible (libadrp has no CPU fallback)");
    if (device < 0 || device >= ndev) return seterr(nullptr, ADRP_ERR_INVALID, "device index out of range");
    adrp_policy_t* p = new adrp_policy_t();
    p->device = device;
    p->in_dim = in_dim; p->h1 = hidden1; p->h2 = hidden2; p->relu = activation == ADRP_POLICY_RELU;
    p->act_dim = act_dim;
    if (const char* env = getenv("ADRP_POLICY_RT")) p->row_tiles = atoi(env);
    const std::vector<float> blob = build_blob(in_dim, hidden1, hidden2, w1, b1, w2, b2, w3, b3, &p->L, act_dim);
    DeviceGuard g(device);
    if (hipMalloc((void**)&p->blob, blob.size() * sizeof(float)) != hipSuccess) {
        delete p;
        return seterr(nullptr, ADRP_ERR_OOM, "hipMalloc failed");
    }
    if (hipMemcpy(p->blob, blob.data(), blob.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
        hipFree(p->blob);
        delete p;
        return seterr(nullptr, ADRP_ERR_DEVICE, "weight upload failed");
    }
    *out = p;
    return ADRP_OK;
}

extern "C" void adrp_policy_destroy(adrp_policy_t* p) {
    if (!p) return;
    DeviceGuard g(p->device);
    hipDeviceSynchronize();
    hipFree(p->blob);
    if (p->critic) hipFree(p->critic);
    if (p->log_std) hipFree(p->log_std);
    delete p;
}

extern "C" int adrp_policy_set_critic(adrp_policy_t* p, const float* vw1, const float* vb1, const float* vw2,
                                      const float* vb2, const float* vw3, const float* vb3, const float* log_std) {
    if (!p || !vw1 || !vb1 || !vw2 || !vb2 || !vw3 || !vb3 || !log_std)
        return seterr(nullptr, ADRP_ERR_INVALID, "adrp_policy_set_critic: NULL argument");
    DeviceGuard g(p->device);
    if (p->critic) { hipFree(p->critic); p->critic = nullptr; }
    if (p->log_std) { hipFree(p->log_std); p->log_std = nullptr; }
    const std::vector<float> blob = build_blob(p->in_dim, p->h1, p->h2, vw1, vb1, vw2, vb2, vw3, vb3, &p->Lc, 1);
    int rc = upload(blob, &p->critic);
    if (rc == ADRP_OK) rc = upload(std::vector<float>(log_std, log_std + p->act_dim), &p->log_std);
    if (rc != ADRP_OK) return seterr(nullptr, rc, "adrp_policy_set_critic: upload failed");
    return ADRP_OK;
}

template <int T1, int T2>
static hipError_t launch_sample(const adrp_policy_t* p, const PolicySampleArgs& a, hipStream_t s) {
    constexpr int NW = T1 > T2 ? T1 : T2;
    const dim3 grid((a.rows + 15) / 16), blk(2 * 64 * NW);
    if (p->relu) hipLaunchKernelGGL((policy_sample_kernel<T1, T2, true>), grid, blk, 0, s, a);
    else hipLaunchKernelGGL((policy_sample_kernel<T1, T2, false>), grid, blk, 0, s, a);
    return hipGetLastError();
}
template <int T1>
static hipError_t sample_t2(const adrp_policy_t* p, const PolicySampleArgs& a, hipStream_t s) {
    switch (p->h2 / 16) {
        case 1: return launch_sample<T1, 1>(p, a, s);
        case 2: return launch_sample<T1, 2>(p, a, s);
        case 4: return launch_sample<T1, 4>(p, a, s);
        default: return launch_sample<T1, 8>(p, a, s);
    }
}

extern "C" int adrp_policy_sample(adrp_policy_t* p, const float* obs_dev, int rows, int obs_stride, int mode,
                                  uint64_t seed, uint32_t counter, float* env_act_dev, float* action_dev,
                                  float* value_dev, float* logprob_dev, float* eps_dev, void* stream) {
    if (!p || !obs_dev || !env_act_dev || !action_dev || !value_dev || !logprob_dev)
        return seterr(nullptr, ADRP_ERR_INVALID, "adrp_policy_sample: NULL argument");
    if (!p->critic) return seterr(nullptr, ADRP_ERR_INVALID, "adrp_policy_sample: no critic (adrp_policy_set_critic)");
    if (rows < 0 || obs_stride < p->in_dim) return seterr(nullptr, ADRP_ERR_INVALID, "adrp_policy_sample: rows / obs_stride");
    if (mode != ADRP_POLICY_RAW && mode != ADRP_POLICY_RELATIVE && mode != ADRP_POLICY_ABSOLUTE)
        return seterr(nullptr, ADRP_ERR_INVALID, "adrp_policy_sample: mode");
    if (mode != ADRP_POLICY_RAW && (p->act_dim != 4 || p->in_dim < 6))
        return seterr(nullptr, ADRP_ERR_INVALID, "RELATIVE / ABSOLUTE need 4 actions (and the pose in obs[0:6])");
    if (rows == 0) return ADRP_OK;
    PolicySampleArgs a;
    a.actor = p->blob; a.La = p->L; a.critic = p->critic; a.Lc = p->Lc; a.log_std = p->log_std;
    a.obs = obs_dev; a.rows = rows; a.obs_stride = obs_stride; a.mode = mode; a.act_dim = p->act_dim;
    a.seed = seed; a.counter = counter;
    a.env_act = env_act_dev; a.action = action_dev; a.value = value_dev; a.log_prob = logprob_dev; a.eps = eps_dev;
    DeviceGuard g(p->device);
    hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    switch (p->h1 / 16) {
        case 1: e = sample_t2<1>(p, a, s); break;
        case 2: e = sample_t2<2>(p, a, s); break;
        case 4: e = sample_t2<4>(p, a, s); break;
        default: e = sample_t2<8>(p, a, s); break;
    }
    if (e != hipSuccess) return seterr(nullptr, ADRP_ERR_DEVICE, std::string("policy sample launch: ") + hipGetErrorString(e));
    return ADRP_OK;
}

extern "C" int adrp_policy_act(adrp_policy_t* p, const float* obs_dev, int rows, int obs_stride, int mode,
                               float* act_dev, void* stream) {
    if (!p || !obs_dev || !act_dev) return seterr(nullptr, ADRP_ERR_INVALID, "adrp_policy_act: NULL argument");
    if (p->act_dim != 4) return seterr(nullptr, ADRP_ERR_INVALID, "adrp_policy_act: 4 actions (adrp_policy_sample takes 1..4)");
    if (rows < 0 || obs_stride < p->in_dim) return seterr(nullptr, ADRP_ERR_INVALID, "adrp_policy_act: rows / obs_stride");
    if (mode != ADRP_POLICY_RAW && mode != ADRP_POLICY_RELATIVE && mode != ADRP_POLICY_ABSOLUTE)
        return seterr(nullptr, ADRP_ERR_INVALID, "adrp_policy_act: mode");
    if (mode == ADRP_POLICY_RELATIVE && p->in_dim < 6)
        return seterr(nullptr, ADRP_ERR_INVALID, "RELATIVE mode reads the pose from obs[0:3] and obs[5]");
    if (rows == 0) return ADRP_OK;
    DeviceGuard g(p->device);
    hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    switch (p->h1 / 16) {
        case 1: e = dispatch_t2<1>(p, obs_dev, rows, obs_stride, act_dev, mode, s); break;
        case 2: e = dispatch_t2<2>(p, obs_dev, rows, obs_stride, act_dev, mode, s); break;
        case 4: e = dispatch_t2<4>(p, obs_dev, rows, obs_stride, act_dev, mode, s); break;
        default: e = dispatch_t2<8>(p, obs_dev, rows, obs_stride, act_dev, mode, s); break;
    }
    if (e != hipSuccess) return seterr(nullptr, ADRP_ERR_DEVICE, std::string("policy launch: ") + hipGetErrorString(e));
    return ADRP_OK;
}

// ---- GAE (SB3 RolloutBuffer.compute_returns_and_advantage) -----------------------------------
// one lane per env walks its n_steps backwards; every [step][env] access is coalesced across the
// wave.  float32 arithmetic with the NumPy expression order (float32 arrays x Python floats).
__global__ void __launch_bounds__(256) gae_kernel(const float* __restrict__ rew, const float* __restrict__ val,
                                                  const float* __restrict__ starts, const float* __restrict__ last_val,
                                                  const float* __restrict__ dones, int T, int E, float gamma, float gl,
                                                  float* __restrict__ adv, float* __restrict__ ret) {
#pragma clang fp contract(off)
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    float last = 0.0f;
    float next_v = last_val[e], next_nt = 1.0f - dones[e];
    for (int t = T - 1; t >= 0; --t) {
        const size_t k = size_t(t) * E + e;
        const float v = val[k];
        const float delta = rew[k] + gamma * next_v * next_nt - v;
        last = delta + gl * next_nt * last;   // gl = float32(gamma * gae_lambda): NumPy multiplies the two Python floats first
        adv[k] = last;
        ret[k] = last + v;
        next_v = v;
        next_nt = 1.0f - starts[k];
    }
}

extern "C" int adrp_gae(const float* rewards, const float* values, const float* episode_starts, const float* last_values,
                        const float* dones, int n_steps, int n_envs, double gamma, double gae_lambda, float* advantages,
                        float* returns, void* stream) {
    if (!rewards || !values || !episode_starts || !last_values || !dones || !advantages || !returns)
        return seterr(nullptr, ADRP_ERR_INVALID, "adrp_gae: NULL argument");
    if (n_steps < 0 || n_envs < 0) return seterr(nullptr, ADRP_ERR_INVALID, "adrp_gae: sizes");
    if (n_steps == 0 || n_envs == 0) return ADRP_OK;
    StreamDeviceGuard g((hipStream_t)stream);
    hipLaunchKernelGGL(gae_kernel, dim3((n_envs + 255) / 256), dim3(256), 0, (hipStream_t)stream, rewards, values,
                       episode_starts, last_values, dones, n_steps, n_envs, float(gamma), float(gamma * gae_lambda), advantages,
                       returns);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return seterr(nullptr, ADRP_ERR_DEVICE, std::string("gae launch: ") + hipGetErrorString(e));
    return ADRP_OK;
}

// ---------------------------------------------------------------------------------------
// SB3 VecEnv host path (vec_env.py): the terminal observations of the envs that finished, gathered
// behind the step's packed outputs so one device -> host copy carries them (DummyVecEnv puts
// infos[e]["terminal_observation"] only on the envs whose episode ended).  One workgroup of 1024
// lanes scans the done flags in 1024-env chunks: wave ballots + per-wave counts in LDS give each
// done env its rank, idx[rank] = env (ascending); then the first min(count, cap) rows are copied.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) compact_rows_kernel(const uint8_t* __restrict__ term,
                                                            const uint8_t* __restrict__ trunc,
                                                            const float* __restrict__ rows, int n, int rf, int cap,
                                                            int32_t* __restrict__ count, int32_t* __restrict__ idx,
                                                            float* __restrict__ out) {
    __shared__ int wsum[16];
    __shared__ int total;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int base = 0;
    for (int c0 = 0; c0 < n; c0 += 1024) {
        const int i = c0 + tid;
        const bool f = i < n && (term[i] | trunc[i]) != 0;
        const uint64_t b = __ballot(f);
        if (lane == 0) wsum[wave] = __popcll(b);
        __syncthreads();
        int off = base, tot = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            const int c = wsum[w];
            off += w < wave ? c : 0;
            tot += c;
        }
        if (f) idx[off + __popcll(b & ((uint64_t(1) << lane) - 1))] = i;
        base += tot;
        __syncthreads();   // wsum is rewritten by the next chunk
    }
    if (tid == 0) {
        count[0] = base;
        total = base;
    }
    __syncthreads();   // idx (global, this workgroup's writes) and total visible to every lane
    const int m = total < cap ? total : cap;
    const long long nf = (long long)m * rf;
    for (long long k = tid; k < nf; k += 1024) {
        const int j = int(k / rf), c = int(k - (long long)j * rf);
        out[k] = rows[(long long)idx[j] * rf + c];
    }
}

extern "C" int adrp_compact_rows(const uint8_t* term, const uint8_t* trunc, const float* rows, int n, int row_floats,
                                 int cap, int32_t* count, int32_t* idx, float* out_rows, void* stream) {
    if (!term || !trunc || !rows || !count || !idx || (cap > 0 && !out_rows))
        return seterr(nullptr, ADRP_ERR_INVALID, "adrp_compact_rows: NULL argument");
    if (n < 0 || row_floats <= 0 || cap < 0) return seterr(nullptr, ADRP_ERR_INVALID, "adrp_compact_rows: sizes");
    StreamDeviceGuard g((hipStream_t)stream);
    hipLaunchKernelGGL(compact_rows_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, term, trunc, rows, n, row_floats,
                       cap, count, idx, out_rows);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return seterr(nullptr, ADRP_ERR_DEVICE, std::string("compact launch: ") + hipGetErrorString(e));
    return ADRP_OK;
}

// adrp_vec_step's compaction (the host block of one step): flags term / trunc / done copied out of the
// device, the finished envs' ids into the device scratch (the row gather reads them from there) and
// the host block, the first min(count, cap) terminal rows into the host block.  Same ranking as
// compact_rows_kernel.
__global__ void __launch_bounds__(1024) vec_compact_kernel(const uint8_t* __restrict__ term, const uint8_t* __restrict__ trunc,
                                                           const float* __restrict__ rows, int n, int rf, int cap,
                                                           uint8_t* __restrict__ term_o, uint8_t* __restrict__ trunc_o,
                                                           uint8_t* __restrict__ done_o, int32_t* __restrict__ count,
                                                           int32_t* __restrict__ idx_dev, int32_t* __restrict__ idx_o,
                                                           float* __restrict__ out) {
    __shared__ int wsum[16];
    __shared__ int total;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int base = 0;
    for (int c0 = 0; c0 < n; c0 += 1024) {
        const int i = c0 + tid;
        const uint8_t te = i < n ? term[i] : 0, tr = i < n ? trunc[i] : 0;
        const bool f = (te | tr) != 0;
        if (i < n) {
            term_o[i] = te;
            trunc_o[i] = tr;
            done_o[i] = f;
        }
        const uint64_t b = __ballot(f);
        if (lane == 0) wsum[wave] = __popcll(b);
        __syncthreads();
        int off = base, tot = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            const int c = wsum[w];
            off += w < wave ? c : 0;
            tot += c;
        }
        if (f) {
            const int r = off + __popcll(b & ((uint64_t(1) << lane) - 1));
            idx_dev[r] = i;
            idx_o[r] = i;
        }
        base += tot;
        __syncthreads();
    }
    if (tid == 0) {
        count[0] = base;
        total = base;
    }
    __syncthreads();
    const int m = total < cap ? total : cap;
    const long long nf = (long long)m * rf;
    for (long long k = tid; k < nf; k += 1024) {
        const int j = int(k / rf), c = int(k - (long long)j * rf);
        out[k] = rows[(long long)idx_dev[j] * rf + c];
    }
}

int vec_compact_launch(const adrp_vec_io& d, int n, int rf, hipStream_t s) {
    hipLaunchKernelGGL(vec_compact_kernel, dim3(1), dim3(1024), 0, s, d.term_dev, d.trunc_dev, d.tobs_dev, n, rf, d.cap,
                       d.term, d.trunc, d.done, d.count, d.idx_dev, d.idx, d.rows);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ADRP_OK : ADRP_ERR_DEVICE;
}

// the host path's copies and wait without a framework dispatch in between (vec_env.py): kind 1 =
// host -> device, 2 = device -> host (pinned host memory: asynchronous on the stream)
extern "C" int adrp_memcpy_async(void* dst, const void* src, size_t bytes, int kind, void* stream) {
    if (!dst || !src || (kind != 1 && kind != 2)) return seterr(nullptr, ADRP_ERR_INVALID, "adrp_memcpy_async: arguments");
    StreamDeviceGuard g((hipStream_t)stream);
    const hipError_t e = hipMemcpyAsync(dst, src, bytes, kind == 1 ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost,
                                        (hipStream_t)stream);
    if (e != hipSuccess) return seterr(nullptr, ADRP_ERR_DEVICE, std::string("memcpy: ") + hipGetErrorString(e));
    return ADRP_OK;
}
extern "C" int adrp_stream_synchronize(void* stream) {
    StreamDeviceGuard g((hipStream_t)stream);
    const hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    if (e != hipSuccess) return seterr(nullptr, ADRP_ERR_DEVICE, std::string("stream sync: ") + hipGetErrorString(e));
    return ADRP_OK;
}
