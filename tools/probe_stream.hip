// Streaming-read probe: how fast can a wave-per-chunk loop read HBM on this
// box, by load structure.  Not part of the product; used to size the scan
// kernels' prefetch.  Build: hipcc --offload-arch=gfx950 -O3 probe_stream.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 v4u __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ v4u ld(const uint8_t *p) {
    return __builtin_nontemporal_load((const v4u *)p);
}

// persistent waves, ticket of SEG bytes, DEPTH-deep ring of 1 KiB per wave
template <int DEPTH, int WAVES>
__global__ void __launch_bounds__(WAVES * 64) ring_probe(const uint8_t *A, u64 n, u64 seg,
                                                          unsigned long long *ticket,
                                                          u32 *sink) {
    const u32 lane = threadIdx.x & 63;
    u32 acc = 0;
    for (;;) {
        unsigned long long t = 0;
        if (lane == 0) t = atomicAdd(ticket, 1ULL);
        t = __shfl(t, 0);
        const u64 lo = t * seg;
        if (lo >= n) break;
        const u32 iters = (u32)(seg >> 10);
        v4u ring[DEPTH];
#pragma unroll
        for (int k = 0; k < DEPTH; k++) ring[k] = ld(A + lo + 1024 * k + 16 * lane);
        for (u32 g = 0; g < iters / DEPTH; g++) {
#pragma unroll
            for (int k = 0; k < DEPTH; k++) {
                v4u v = ring[k];
                acc ^= v.x + v.y * 3 + v.z * 5 + v.w * 7;
                u64 it = (u64)g * DEPTH + k + DEPTH;
                u64 off = it < iters ? lo + 1024 * it : lo;
                ring[k] = ld(A + off + 16 * lane);
            }
        }
    }
    if (acc == 0x12345678) sink[0] = acc;
}

// static segment assignment: wave w takes segments w, w + W, ... (W = all
// waves); each segment SEG bytes read through a DEPTH-deep 1 KiB ring
template <int DEPTH>
__global__ void __launch_bounds__(1024) static_probe(const uint8_t *A, u64 n, u64 seg,
                                                     u32 *sink) {
    const u32 lane = threadIdx.x & 63;
    const u64 W = (u64)gridDim.x * 16;
    const u64 w = (u64)blockIdx.x * 16 + (threadIdx.x >> 6);
    u32 acc = 0;
    const u32 iters = (u32)(seg >> 10);
    for (u64 sg = w; sg * seg < n; sg += W) {
        const u64 lo = sg * seg;
        v4u ring[DEPTH];
#pragma unroll
        for (int k = 0; k < DEPTH; k++) ring[k] = ld(A + lo + 1024 * (k % iters) + 16 * lane);
        for (u32 g = 0; g < (iters + DEPTH - 1) / DEPTH; g++) {
#pragma unroll
            for (int k = 0; k < DEPTH; k++) {
                v4u v = ring[k];
                acc ^= v.x + v.y * 3 + v.z * 5 + v.w * 7;
                u64 it = (u64)g * DEPTH + k + DEPTH;
                u64 off = it < iters ? lo + 1024 * it : lo;
                ring[k] = ld(A + off + 16 * lane);
            }
        }
    }
    if (acc == 0x12345678) sink[0] = acc;
}

// grid-stride, one 16-B load per lane per step, UNROLL independent steps
template <int UNROLL>
__global__ void __launch_bounds__(256) stride_probe(const uint8_t *A, u64 n, u32 *sink) {
    u32 acc = 0;
    const u64 stride = (u64)gridDim.x * 256 * 16;
    for (u64 p = ((u64)blockIdx.x * 256 + threadIdx.x) * 16; p + (UNROLL - 1) * stride < n;
         p += stride * UNROLL) {
        v4u v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) v[u] = ld(A + p + u * stride);
#pragma unroll
        for (int u = 0; u < UNROLL; u++) acc ^= v[u].x + v[u].y * 3 + v[u].z * 5 + v[u].w * 7;
    }
    if (acc == 0x12345678) sink[0] = acc;
}

int main() {
    const u64 n = 4ull << 30;
    uint8_t *A;
    u32 *sink;
    unsigned long long *ticket;
    CHECK(hipMalloc(&A, n));
    CHECK(hipMemset(A, 1, n));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMalloc(&ticket, 8));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto launch) {
        float best = 1e9f;
        for (int r = 0; r < 6; r++) {
            hipMemset(ticket, 0, 8);
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (r > 0 && ms < best) best = ms;
        }
        printf("%-40s %8.3f ms %8.1f GB/s\n", name, best, n / (best * 1e-3) / 1e9);
    };
    const u64 seg = 64 << 10;
    timeit("ring depth 4, 16 waves/WG, 1 WG/CU", [&] {
        hipLaunchKernelGGL((ring_probe<4, 16>), dim3(cus), dim3(1024), 0, 0, A, n, seg, ticket, sink); });
    timeit("ring depth 8, 16 waves/WG, 1 WG/CU", [&] {
        hipLaunchKernelGGL((ring_probe<8, 16>), dim3(cus), dim3(1024), 0, 0, A, n, seg, ticket, sink); });
    timeit("ring depth 4, 16 waves/WG, 2 WG/CU", [&] {
        hipLaunchKernelGGL((ring_probe<4, 16>), dim3(2 * cus), dim3(1024), 0, 0, A, n, seg, ticket, sink); });
    timeit("ring depth 8, 8 waves/WG, 4 WG/CU", [&] {
        hipLaunchKernelGGL((ring_probe<8, 8>), dim3(4 * cus), dim3(512), 0, 0, A, n, seg, ticket, sink); });
    timeit("ring depth 2, 16 waves/WG, 1 WG/CU", [&] {
        hipLaunchKernelGGL((ring_probe<2, 16>), dim3(cus), dim3(1024), 0, 0, A, n, seg, ticket, sink); });
    for (u64 sg : {4096ull, 16384ull, 65536ull}) {
        char nm[80];
        snprintf(nm, sizeof nm, "static seg %llu KiB ring 4, 1 WG/CU", (unsigned long long)(sg >> 10));
        timeit(nm, [&] {
            hipLaunchKernelGGL((static_probe<4>), dim3(cus), dim3(1024), 0, 0, A, n, sg, sink); });
    }
    timeit("ticket seg 16 KiB ring 4, 1 WG/CU", [&] {
        hipLaunchKernelGGL((ring_probe<4, 16>), dim3(cus), dim3(1024), 0, 0, A, n, 16384ull, ticket, sink); });
    timeit("stride unroll 1, 8 WG/CU", [&] {
        hipLaunchKernelGGL((stride_probe<1>), dim3(8 * cus), dim3(256), 0, 0, A, n, sink); });
    timeit("stride unroll 4, 8 WG/CU", [&] {
        hipLaunchKernelGGL((stride_probe<4>), dim3(8 * cus), dim3(256), 0, 0, A, n, sink); });
    timeit("stride unroll 4, 4 WG/CU", [&] {
        hipLaunchKernelGGL((stride_probe<4>), dim3(4 * cus), dim3(256), 0, 0, A, n, sink); });
    return 0;
}
