// Probe (GPU box): does a failed or not-ready HIP call stay the thread's
// last error across later successful calls?  Decides whether a launch
// check (hipGetLastError after hipLaunchKernelGGL) can see a stale error.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void spin(unsigned long long n) {
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < n) {
    }
}
int main() {
    int v = 0;
    hipError_t a = hipSetDevice(99);
    hipError_t b = hipRuntimeGetVersion(&v);
    hipError_t c = hipGetLastError();
    printf("failed call then success: last=%d (%s)\n", c, hipGetErrorString(c));
    hipSetDevice(0);
    hipEvent_t e;
    hipEventCreate(&e);
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, 0, 2000000ULL); // ~20 ms
    hipEventRecord(e, 0);
    hipError_t q = hipEventQuery(e);
    float ms = 0;
    hipEvent_t e0;
    hipEventCreate(&e0);
    hipError_t et = hipEventElapsedTime(&ms, e0, e);
    hipError_t d = hipGetLastError();
    printf("eventQuery=%d elapsedTime(unrecorded/not ready)=%d last=%d (%s)\n", q, et, d,
           hipGetErrorString(d));
    hipDeviceSynchronize();
    (void)a; (void)b;
    return 0;
}
