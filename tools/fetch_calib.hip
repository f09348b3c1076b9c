// fetch_calib.hip — calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths
// the step kernels use (MI355X_MICROARCH.md, HBM: "Other access widths are uncalibrated: calibrate on
// a known byte count in your own access pattern").  Each kernel streams a 256 MiB buffer once per
// launch (beyond the per-XCD L2, so nothing is re-served from L2 across launches) with one element
// per lane per iteration, coalesced: 4 B (the fp32 SoA state fields), 8 B (fp64 fields), 16 B.
// Bytes per launch are printed; tools/pmc_summary.py --calib turns the counter runs into ratios.
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>

template <typename T>
__device__ __forceinline__ float lsum(T v) { return float(v); }
template <>
__device__ __forceinline__ float lsum<float4>(float4 v) { return v.x + v.y + v.z + v.w; }

#define RD(NAME, T)                                                                           \
    __global__ void __launch_bounds__(256) NAME(const T* __restrict__ in, float* out, size_t n) { \
        float acc = 0.0f;                                                                     \
        for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) \
            acc += lsum(in[i]);                                                               \
        if (acc == 1234.5f) out[0] = acc;                                                     \
    }
RD(calib_read4, float)
RD(calib_read8, double)
RD(calib_read16, float4)

#define WR(NAME, T, V)                                                                        \
    __global__ void __launch_bounds__(256) NAME(T* __restrict__ o, size_t n) {                \
        for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) \
            o[i] = V;                                                                         \
    }
WR(calib_write4, float, float(i))
WR(calib_write8, double, double(i))
WR(calib_write16, float4, make_float4(float(i), 0.f, 1.f, 2.f))

int main() {
    const size_t bytes = size_t(256) << 20;
    void* buf = nullptr;
    float* out = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc((void**)&out, 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, bytes);
    const dim3 grid(2048), blk(256);
    for (int r = 0; r < 12; ++r) {
        hipLaunchKernelGGL(calib_read4, grid, blk, 0, 0, (const float*)buf, out, bytes / 4);
        hipLaunchKernelGGL(calib_read8, grid, blk, 0, 0, (const double*)buf, out, bytes / 8);
        hipLaunchKernelGGL(calib_read16, grid, blk, 0, 0, (const float4*)buf, out, bytes / 16);
        hipLaunchKernelGGL(calib_write4, grid, blk, 0, 0, (float*)buf, bytes / 4);
        hipLaunchKernelGGL(calib_write8, grid, blk, 0, 0, (double*)buf, bytes / 8);
        hipLaunchKernelGGL(calib_write16, grid, blk, 0, 0, (float4*)buf, bytes / 16);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"bytes_per_launch\": %zu, \"launches_per_kernel\": 12}\n", bytes);
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}
