// devmap_probe.hip (tools only): can the host write device memory directly (large-BAR mapping), for
// a persistent-step mailbox in HBM?  Allocates fine-grained and coarse-grained device memory, prints
// hipPointerGetAttributes, and only if a host pointer is reported writes it from the CPU and reads it
// back from a kernel.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void readk(const volatile int* p, int* out) { out[0] = p[0]; out[1] = p[1]; }

static void probe(const char* name, unsigned flags) {
    int* d = nullptr;
    hipError_t e = flags ? hipExtMallocWithFlags((void**)&d, 4096, flags) : hipMalloc((void**)&d, 4096);
    if (e != hipSuccess) { printf("%s: alloc failed %s\n", name, hipGetErrorString(e)); return; }
    hipPointerAttribute_t a;
    e = hipPointerGetAttributes(&a, d);
    printf("%s: dev %p attr rc %d type %d devicePointer %p hostPointer %p isManaged %d allocationFlags %u\n", name, (void*)d,
           (int)e, (int)a.type, a.devicePointer, a.hostPointer, (int)a.isManaged, a.allocationFlags);
    if (e == hipSuccess && a.hostPointer) {
        volatile int* h = (volatile int*)a.hostPointer;
        h[0] = 1234; h[1] = 5678;
        int* out; hipMalloc((void**)&out, 8);
        hipLaunchKernelGGL(readk, dim3(1), dim3(1), 0, 0, (const volatile int*)d, out);
        int r[2] = {0, 0};
        hipMemcpy(r, out, 8, hipMemcpyDeviceToHost);
        printf("%s: host wrote 1234 5678, kernel read %d %d, host reads back %d\n", name, r[0], r[1], h[0]);
        hipFree(out);
    }
    hipFree(d);
}

int main() {
    probe("hipMalloc", 0);
    probe("finegrained", hipDeviceMallocFinegrained);
    probe("uncached", hipDeviceMallocUncached);
    return 0;
}
