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
    int in_dim = 0, h1 = 0, h2 = 0, relu = 0;
    int row_tiles = 0;       // 16-row tiles per block (ADRP_POLICY_RT; 0 = default)
    PolicyLayout L{};
    float* blob = nullptr;   // device fragment blob
};

// Pre-permute the Linear weights (torch layout [out][in], row-major) into the per-lane MFMA
// fragments policy_kernel reads (see policy_kernel.h for the k order).
static std::vector<float> build_blob(int in_dim, int H1, int H2, const float* w1, const float* b1, const float* w2,
                                     const float* b2, const float* w3, const float* b3, PolicyLayout* L) {
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
                v[L->f3 + (u * 4 + i) * 64 + l] = out < 4 ? w3[size_t(out) * H2 + k] : 0.0f;
            }
    memcpy(&v[L->b1], b1, sizeof(float) * H1);
    memcpy(&v[L->b2], b2, sizeof(float) * H2);
    memcpy(&v[L->b3], b3, sizeof(float) * 4);
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
    if (!out) return seterr(nullptr, ADRP_ERR_INVALID, "out is NULL");
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
    if (const char* env = getenv("ADRP_POLICY_RT")) p->row_tiles = atoi(env);
    const std::vector<float> blob = build_blob(in_dim, hidden1, hidden2, w1, b1, w2, b2, w3, b3, &p->L);
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
    delete p;
}

extern "C" int adrp_policy_act(adrp_policy_t* p, const float* obs_dev, int rows, int obs_stride, int mode,
                               float* act_dev, void* stream) {
    if (!p || !obs_dev || !act_dev) return seterr(nullptr, ADRP_ERR_INVALID, "adrp_policy_act: NULL argument");
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
