// Issue-rate probe (not part of the product): cycles per wave-instruction
// per SIMD for the integer VALU ops the FDR sweep uses and for random LDS
// reads of each width, with one 1024-thread workgroup per CU (16 waves, 4
// per SIMD) as in vsa_lit_scan.  Build:
//   hipcc --offload-arch=gfx950 -O3 tools/probe_issue.hip -o tools/probe_issue
// Output: one line per probe, ns per launch and cycles per wave-instruction
// per SIMD at the clock measured in-kernel (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 v4u __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define ITERS 4096

// 32 independent chains of one op kind; 32 ops per loop trip
template <int OP>
__global__ void __launch_bounds__(1024) valu_probe(u32 *sink, u64 *clk, u32 seed) {
    u32 a[32];
#pragma unroll
    for (int i = 0; i < 32; i++) a[i] = threadIdx.x * 2654435761u + i * seed;
    const u32 s = seed | 1;
    u64 t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 32; i++) {
            u32 x = a[i], y = a[(i + 1) & 31];
            if constexpr (OP == 0) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "s"(s));
            if constexpr (OP == 1) asm volatile("v_alignbyte_b32 %0, %0, %1, 3" : "+v"(x) : "v"(y));
            if constexpr (OP == 2) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(x) : "s"(s), "v"(y));
            if constexpr (OP == 3) asm volatile("v_mad_u32_u16 %0, %0, 4, %1 op_sel:[1,0,0,0]" : "+v"(x) : "s"(s));
            if constexpr (OP == 4) asm volatile("v_pk_lshrrev_b16 %0, %1, %0" : "+v"(x) : "s"(s));
            if constexpr (OP == 5) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "s"(s));
            if constexpr (OP == 6) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 bound_ctrl:0" : "+v"(x) : "v"(y));
            if constexpr (OP == 7) asm volatile("v_or_b32 %0, %0, %1" : "+v"(x) : "v"(y));
            if constexpr (OP == 8) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(y));
            if constexpr (OP == 9) asm volatile("v_cmp_ne_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(y) : "vcc");
            if constexpr (OP == 10) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x));
            if constexpr (OP == 11) asm volatile("v_and_b32 %0, %1, %0" : "+v"(x) : "s"(s));
            if constexpr (OP == 12) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(x) : "v"(y));
            if constexpr (OP == 13) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "s"(s), "v"(y));
            if constexpr (OP == 14) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "s"(s));
            if constexpr (OP == 15) asm volatile("v_or_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "+v"(x) : "v"(y));
            if constexpr (OP == 16) asm volatile("v_or_b32_dpp %0, %1, %0 row_shr:1 bound_ctrl:0" : "+v"(x) : "v"(y));
            if constexpr (OP == 17) asm volatile("v_bfe_u32 %0, %0, 8, 7" : "+v"(x));
            if constexpr (OP == 18) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "s"(s));
            if constexpr (OP == 19) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(x) : "s"(s));
            if constexpr (OP == 20) asm volatile("v_or_b32 %0, %1, %0" : "+v"(x) : "s"(s));
            if constexpr (OP == 21) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(y));
            if constexpr (OP == 22) asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 bound_ctrl:0" : "+v"(x) : "v"(y));
            if constexpr (OP == 23) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(x) : "s"(s));
            if constexpr (OP == 24) asm volatile("v_alignbit_b32 %0, %0, %1, 9" : "+v"(x) : "v"(y));
            if constexpr (OP == 25) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(y));
            if constexpr (OP == 26) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(y));
            if constexpr (OP == 27) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(y));
            a[i] = x;
        }
    }
    u64 t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    u32 acc = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) acc ^= a[i];
    if (acc == 0x12345678u) sink[0] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

// random LDS reads: W bytes per lane per read (4, 8, 16) at 16 fixed
// random addresses per lane (a real address in `pct` % of the lanes, the
// others all read address 0: a broadcast), one v_xor per read; volatile
// loads keep the width
template <int W, bool CONFLICT_FREE>
__global__ void __launch_bounds__(1024) lds_probe(u32 *sink, u64 *clk, u32 seed, u32 nbytes,
                                                  u32 pct) {
    extern __shared__ u32 tab[];
    for (u32 i = threadIdx.x; i < nbytes / 4; i += 1024) tab[i] = i * 2654435761u ^ seed;
    __syncthreads();
    const u32 lane = threadIdx.x & 63;
    u32 ad[16];
    const u32 amask = (nbytes - 1) & ~(u32)(W - 1);
#pragma unroll
    for (int i = 0; i < 16; i++) {
        u32 h = (threadIdx.x * 7919u + i * 104729u + seed) * 2654435761u;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        u32 a = (h * W) & amask;
        if (CONFLICT_FREE) a = (a & ~(u32)(32 * W - 1)) | ((lane & 31) * W);
        if ((h >> 24) % 100 >= pct) a = 0;
        ad[i] = a;
    }
    u32 acc[16];
#pragma unroll
    for (int i = 0; i < 16; i++) acc[i] = 0;
    u64 t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS / 4; it++) {
        if constexpr (W == 4) {
            u32 r[16];
#pragma unroll
            for (int i = 0; i < 16; i++) asm volatile("ds_read_b32 %0, %1" : "=v"(r[i]) : "v"(ad[i]));
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15]));
#pragma unroll
            for (int i = 0; i < 16; i++) acc[i] ^= r[i];
        } else if constexpr (W == 8) {
            u64 r[16];
#pragma unroll
            for (int i = 0; i < 16; i++) asm volatile("ds_read_b64 %0, %1" : "=v"(r[i]) : "v"(ad[i]));
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15]));
#pragma unroll
            for (int i = 0; i < 16; i++) acc[i] ^= (u32)r[i];
        } else {
            v4u r[16];
#pragma unroll
            for (int i = 0; i < 16; i++) asm volatile("ds_read_b128 %0, %1" : "=v"(r[i]) : "v"(ad[i]));
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15]));
#pragma unroll
            for (int i = 0; i < 16; i++) acc[i] ^= r[i].x;
        }
    }
    u64 t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    u32 x = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) x ^= acc[i];
    if (x == 0x12345678u) sink[0] = x;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    u32 *sink;
    u64 *clk, hclk[2];
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMalloc(&clk, 16));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto run = [&](const char *name, double instr_per_wave, auto launch) {
        float best = 1e9f;
        for (int r = 0; r < 8; r++) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (r > 1 && ms < best) best = ms;
        }
        hipMemcpy(hclk, clk, 16, hipMemcpyDeviceToHost);
        const double ghz = (double)hclk[0] / ((double)hclk[1] * 10.0);  // memrealtime = 100 MHz
        const double cyc = (double)hclk[0];
        // 16 waves per CU on 4 SIMDs: 4 waves per SIMD issue instr_per_wave each
        printf("{\"probe\": \"%s\", \"ms\": %.4f, \"ghz\": %.3f, \"wave0_cyc_per_instr\": %.3f, "
               "\"wall_cyc_per_instr_per_simd\": %.3f}\n",
               name, best, ghz, cyc / instr_per_wave, best * 1e-3 * ghz * 1e9 / (instr_per_wave * 4.0));
        fflush(stdout);
    };
    const char *vnames[] = {"v_or3_b32", "v_alignbyte_b32", "v_bfi_b32", "v_mad_u32_u16",
                            "v_pk_lshrrev_b16", "v_perm_b32", "v_mov_b32_dpp", "v_or_b32",
                            "v_add_u32", "v_cmp+v_cndmask(2)", "v_lshlrev_b32", "v_and_b32(s)",
                            "v_lshl_or_b32", "v_and_or_b32", "v_add3_u32", "v_or_b32_sdwa",
                            "v_or_b32_dpp", "v_bfe_u32", "v_fma_f32", "v_lshrrev_b32(s)",
                            "v_or_b32(s)", "v_cndmask_b32", "v_mov_dpp_wave_shr", "v_lshl_add_u32",
                            "v_alignbit_b32", "v_pk_add_u16", "v_xor_b32", "v_mul_u32_u24"};
    const double vinstr = 32.0 * ITERS;
#define VP(OP) run(vnames[OP], (OP == 9 ? 2.0 : 1.0) * vinstr, [&] { \
        valu_probe<OP><<<cus, 1024>>>(sink, clk, 12345u); })
    VP(0); VP(1); VP(2); VP(3); VP(4); VP(5); VP(6); VP(7); VP(8); VP(9);
    VP(10); VP(11); VP(12); VP(13); VP(14); VP(15); VP(16); VP(17); VP(18); VP(19);
    VP(20); VP(21); VP(22); VP(23); VP(24); VP(25); VP(26); VP(27);
    const double linstr = 16.0 * (ITERS / 4);
    const u32 nb = 128u << 10;
    // LDS rows: wall cycles are per CU (16 waves share one LDS): report
    // cycles per wave-instruction per CU = wall / (16 waves x instr)
    auto lrun = [&](const char *name, auto launch) {
        float best = 1e9f;
        for (int r = 0; r < 8; r++) {
            (void)hipEventRecord(e0);
            launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (r > 1 && ms < best) best = ms;
        }
        (void)hipMemcpy(hclk, clk, 16, hipMemcpyDeviceToHost);
        const double ghz = (double)hclk[0] / ((double)hclk[1] * 10.0);
        printf("{\"probe\": \"%s\", \"ms\": %.4f, \"ghz\": %.3f, \"lds_cyc_per_instr_per_cu\": %.3f}\n",
               name, best, ghz, best * 1e-3 * ghz * 1e9 / (linstr * 16.0));
        fflush(stdout);
    };
    char nm[64];
    for (u32 pct : {100u, 50u, 28u, 0u}) {
        snprintf(nm, sizeof nm, "lds_b32_random_%u", pct);
        lrun(nm, [&] { lds_probe<4, false><<<cus, 1024, nb>>>(sink, clk, 7u, nb, pct); });
        snprintf(nm, sizeof nm, "lds_b64_random_%u", pct);
        lrun(nm, [&] { lds_probe<8, false><<<cus, 1024, nb>>>(sink, clk, 7u, nb, pct); });
        snprintf(nm, sizeof nm, "lds_b128_random_%u", pct);
        lrun(nm, [&] { lds_probe<16, false><<<cus, 1024, nb>>>(sink, clk, 7u, nb, pct); });
    }
    lrun("lds_b32_confree", [&] { lds_probe<4, true><<<cus, 1024, nb>>>(sink, clk, 7u, nb, 100u); });
    lrun("lds_b64_confree", [&] { lds_probe<8, true><<<cus, 1024, nb>>>(sink, clk, 7u, nb, 100u); });
    lrun("lds_b128_confree", [&] { lds_probe<16, true><<<cus, 1024, nb>>>(sink, clk, 7u, nb, 100u); });
    return 0;
}
