/*
 * kernels.hip — MI355X (gfx950) kernels for the Vectorscan literal /
 * char-class prefilter hot path.
 *
 *  vsa_lit_scan<MODE>  FDR (fdr.c:145-333) and Teddy / Fat Teddy
 *                      (teddy.c:921-1066, teddy_avx2.c:395-706): first-stage
 *                      filter + exact confirm (fdr_confirm_runtime.h:43-102)
 *                      in one pass.
 *                      Noodle (noodle_engine.cpp:75-134) is a fourth mode
 *                      of the same kernel (masked compare, no table).
 *  vsa_class_scan      shufti / truffle / vermicelli reduced to a 256-bit
 *                      byte class (shufti_simd.hpp:89-280, x86/truffle.hpp,
 *                      vermicelli_simd.cpp) -> 1 bit/byte bitmap + first/last.
 *
 * Work decomposition (literal scan): the batch is a list of blocks (each one
 * hwlmExec call) cut into segments by the host (runtime.hip build_plan);
 * workgroup b owns a list of segments holding an equal share of the bytes
 * and its scanning waves take them in turn from an LDS counter, sweeping
 * each in 1 KiB iterations: lane l loads 16 bytes at iteration_base + 16 l
 * with one global_load_dwordx4 (fully coalesced), so HBM is read once plus
 * a 1 KiB-aligned halo per segment.
 *
 * FDR / Teddy filter (the reference's stride-1 shift-or, restated per lane):
 * for end e, conf(e) = OR_k field_k(T[key(e-k)]); a zero bit b means
 * "bucket b may end here".  Each lane walks its 16 positions keeping a
 * running state S (S |= T[key(p)]; conf(p) = low field; S >>= field width);
 * the spill into the next lane's first ends travels by one wave shuffle
 * (S_out -> S_in of lane+1, lane 63 -> next iteration's lane 0).  Tables
 * live in LDS: the FDR domain table as-is (2^d x 8 B), Teddy's nibble
 * masks pre-combined per byte value and replicated 32x so that the lane
 * group's 32 random lookups hit 32 distinct banks.
 *
 * Candidates (rare) are compacted per wave into an LDS queue with a wave
 * prefix sum and confirmed 64 at a time, one per lane: mul-hash of the 8
 * bytes ending at e, litIndex lookup, LitInfo chain walk, overhang check.
 * Confirmed matches are appended with a sort key that reproduces the
 * reference callback order (kernels.h).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

#define WAVE 64
#define LIT_WAVES 16
/* diagnostics that touch the hot loops (candidate-path cycles, the confirm
 * wave's end phase) exist only in -DVSA_DIAG builds
 * (tools/build_variant.sh diag -DVSA_DIAG): measured 1-2 % on the cfg-4
 * scan even when off (profiles/r05/r05u_*) */
#ifdef VSA_DIAG
#define VSA_DIAG_ON 1
#else
#define VSA_DIAG_ON 0
#endif
/* an experiment hook of the candidate / confirm paths (VSA_DEBUG_FLAGS
 * bits: 8 filter only, 16 drop expanded candidates, 32 count first-stage
 * candidates, 64 confirm-wave phase profile, 128 drop gathered entries, 256
 * short ring entries, 1024 no confirm-wave priority): compiled out of
 * product builds, so the hot paths test no flag word (tools/build_variant.sh
 * diag -DVSA_DIAG builds the library with them) */
#define VSA_DBG(flags, bits) (VSA_DIAG_ON && ((flags) & (bits)))
#define LIT_THREADS (LIT_WAVES * WAVE)
#define QCAP 256

typedef uint32_t u32;
typedef uint64_t u64;
typedef uint8_t u8;

__device__ __forceinline__ u32 lane_id() { return __lane_id(); }

/* the builtins return int: keep them unsigned so u64 assembly never
 * sign-extends a low word */
__device__ __forceinline__ u32 readlane_u32(u32 v, int src) {
    return (u32)__builtin_amdgcn_readlane((int)v, src);
}
__device__ __forceinline__ u32 readfirstlane_u32(u32 v) {
    return (u32)__builtin_amdgcn_readfirstlane((int)v);
}

__device__ __forceinline__ u32 shfl_u32(u32 v, int src) {
    return (u32)__shfl((int)v, src, WAVE);
}
__device__ __forceinline__ u32 shfl_up_u32(u32 v, unsigned d) {
    return (u32)__shfl_up((int)v, d, WAVE);
}
/* whole-wave shift by one lane through DPP (no LDS traffic): up1 gives lane
 * l the value of lane l-1 (lane 0 gets 0), down1 that of lane l+1 (lane 63
 * gets 0) */
__device__ __forceinline__ u32 lane_up1(u32 v) {
    return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, true);
}
__device__ __forceinline__ u32 lane_down1(u32 v) {
    return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, true);
}
/* lane l gets lane l-1's v, lane 0 keeps old (wave_shr:1 with the
 * out-of-range lane disabled): one v_mov_dpp */
__device__ __forceinline__ u32 lane_up1_or_old(u32 old, u32 v) {
    return (u32)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xf, 0xf, false);
}
/* lane l gets lane l-1's v, lane 0 lane 63's (wave_ror:1) */
__device__ __forceinline__ u32 lane_ror1(u32 v) {
    return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x13c, 0xf, 0xf, true);
}
/* v with lane `l` replaced by the wave-uniform s (v_writelane) */
template <int L>
__device__ __forceinline__ u32 writelane_u32(u32 v, u32 s) {
    /* s is wave-uniform; readfirstlane pins it to an SGPR (free when it is
     * one already) */
    asm("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(readfirstlane_u32(s)), "n"(L));
    return v;
}
typedef const __attribute__((address_space(3))) u64 lds_u64_t;
typedef const __attribute__((address_space(3))) u8 lds_u8_t;
__device__ __forceinline__ u64 lds_ld64(u32 addr) { return *(lds_u64_t *)(uintptr_t)addr; }

/* Teddy tables live at this LDS byte address (64 KiB; rings and slot
 * bitmaps below it) */
#define TEDDY_TAB_LDS 0x10000u

/* three-input OR in one VALU op (the backend re-associates wide OR trees
 * into two-input ORs) */
__device__ __forceinline__ u32 or3(u32 a, u32 b, u32 c) {
    u32 r;
    asm("v_or3_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ u32 shfl_xor_u32(u32 v, int m) {
    return (u32)__shfl_xor((int)v, m, WAVE);
}
__device__ __forceinline__ u32 shfl_down_u32(u32 v, unsigned d) {
    return (u32)__shfl_down((int)v, d, WAVE);
}
/* lane l gets lane l ^ M's v for a constant M, without the LDS crossbar
 * where CDNA's DPP reaches: xor 1 / 2 are quad permutes, xor 4 = the
 * half-row mirror (l ^ 7) then the quad reverse (^ 3), xor 8 = the row
 * mirror (^ 15) then the half-row mirror (^ 7); xor 16 a ds_swizzle in
 * bit mode (32-lane groups, no address VGPR); xor 32 a bpermute */
template <int M>
__device__ __forceinline__ u32 lane_xor(u32 v) {
    static_assert(M == 1 || M == 2 || M == 4 || M == 8 || M == 16 || M == 32, "lane_xor");
    if constexpr (M == 1) {
        return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);
    } else if constexpr (M == 2) {
        return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);
    } else if constexpr (M == 4) {
        const int h = __builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false);
        return (u32)__builtin_amdgcn_update_dpp(0, h, 0x1B, 0xf, 0xf, false);
    } else if constexpr (M == 8) {
        const int h = __builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, false);
        return (u32)__builtin_amdgcn_update_dpp(0, h, 0x141, 0xf, 0xf, false);
    } else if constexpr (M == 16) {
        return (u32)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);
    } else {
        return shfl_xor_u32(v, 32);
    }
}

/* A wave's 4 sort bins (the binned sort's unit, vsa_bin_finish and the
 * fused finish): bin j holds m[j] <= VSA_SORT_BIN_MAX records at staging row
 * row0 + j.  One register bitonic network of S lanes per bin (S = the next
 * power of two >= the largest count, 2..64), 64 / S bins per pass, npass
 * passes run in lockstep.  Lane r of a bin's S lanes ends up with the bin's
 * r-th smallest key (keys are unique: end, bucket, LitInfo -- the full
 * sort's order); ok[p] says it is a record. */
struct Bins4 {
    u64 k[4];
    u32 id[4], jb[4];
    bool ok[4];
    u32 S, npass, r;
};
/* every pass's loads issued together.  Unconditional (an address inside
 * the wave's 4 bins for every lane, the unused ones masked at the sort): a
 * load under a divergent branch makes the compiler wait for it early */
__device__ __forceinline__ void bins4_load(Bins4 &B, const uint64_t *skeys, const uint32_t *sids,
                                           size_t row0, const u32 (&m)[4], bool sorting,
                                           u32 lane) {
    u32 mmax = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) mmax = m[j] > mmax ? m[j] : mmax;
    B.S = 2;
    while (B.S < mmax && B.S < WAVE) B.S <<= 1;
    const u32 per = WAVE / B.S; /* bins per pass (1..32; >= 4 covers all 4 in one) */
    B.npass = (4 + per - 1) / per; /* wave-uniform, 1..4 */
    const u32 j_l = lane / B.S;
    B.r = lane % B.S;
#pragma unroll
    for (u32 p = 0; p < 4; p++) {
        const u32 j = p * per + j_l;
        B.jb[p] = j;
        const u32 mj = j == 0 ? m[0] : j == 1 ? m[1] : j == 2 ? m[2] : j == 3 ? m[3] : 0u;
        B.ok[p] = sorting && p * per < 4 && B.r < mj;
        const size_t q = (row0 + (j & 3)) * VSA_SORT_BIN_MAX + B.r;
        B.k[p] = skeys[q];
        B.id[p] = sids[q];
    }
}
/* the passes' networks in lockstep (independent exchanges issued together),
 * each step's partner fetched with lane_xor at a constant stride: DPP for
 * strides <= 8, a swizzle for 16, a bpermute only for 32 (S = 64).  Empty
 * slots hold ~0 and sort to the end of their bin. */
__device__ __forceinline__ void bins4_sort(Bins4 &B, u32 lane) {
#pragma unroll
    for (u32 p = 0; p < 4; p++) {
        if (!B.ok[p]) {
            B.k[p] = ~0ULL;
            B.id[p] = 0u;
        }
    }
    const u32 S = B.S, npass = B.npass;
    auto step = [&](auto jc, u32 size) {
        constexpr int JJ = decltype(jc)::value;
        /* ascending within each S-lane segment: the last merge is ascending
         * everywhere, earlier ones alternate */
        const bool up = size == S || (lane & size) == 0;
        const bool lower = (lane & JJ) == 0;
#pragma unroll
        for (u32 p = 0; p < 4; p++) {
            if (p >= npass) break; /* wave-uniform */
            const u32 plo = lane_xor<JJ>((u32)B.k[p]);
            const u32 phi = lane_xor<JJ>((u32)(B.k[p] >> 32));
            const u32 pid = lane_xor<JJ>(B.id[p]);
            const u64 pkk = ((u64)phi << 32) | plo;
            const bool take = (lower == up) ? (pkk < B.k[p]) : (pkk > B.k[p]);
            if (take) {
                B.k[p] = pkk;
                B.id[p] = pid;
            }
        }
    };
    using std::integral_constant;
    for (u32 size = 2; size <= S; size <<= 1) {
        /* a merge of `size`: strides size / 2 .. 1 (wave-uniform branches) */
        if (size >= 64) step(integral_constant<int, 32>(), size);
        if (size >= 32) step(integral_constant<int, 16>(), size);
        if (size >= 16) step(integral_constant<int, 8>(), size);
        if (size >= 8) step(integral_constant<int, 4>(), size);
        if (size >= 4) step(integral_constant<int, 2>(), size);
        step(integral_constant<int, 1>(), size);
    }
}
/* The fused finish's form of bins4_load: a wave's nbins <= 16 consecutive
 * bins (counts cnt[0..nbins) in LDS, all <= S <= 64), 64 / S bins per pass;
 * this loads passes [pass0, pass0 + 4) of them (B.npass of which exist). */
__device__ __forceinline__ void bins16_load(Bins4 &B, const uint64_t *skeys, const uint32_t *sids,
                                            size_t row0, const u32 *cnt, u32 nbins, u32 S,
                                            u32 pass0, u32 lane) {
    B.S = S;
    const u32 per = WAVE / S;
    const u32 np = (nbins + per - 1) / per; /* passes in all (wave-uniform) */
    B.npass = np > pass0 ? (np - pass0 < 4 ? np - pass0 : 4u) : 0u;
    const u32 j_l = lane / S;
    B.r = lane % S;
#pragma unroll
    for (u32 p = 0; p < 4; p++) {
        const u32 j = (pass0 + p) * per + j_l;
        const u32 jc = j < nbins ? j : nbins - 1;
        B.jb[p] = j;
        B.ok[p] = p < B.npass && j < nbins && B.r < cnt[jc];
        const size_t q = (row0 + jc) * VSA_SORT_BIN_MAX + B.r;
        B.k[p] = skeys[q];
        B.id[p] = sids[q];
    }
}

/* the sorted records to their positions: bin j's first at off[j] (and into
 * the packed collective buffer [header | keys (pk_cap) | ids], if any) */
__device__ __forceinline__ void bins4_write(const Bins4 &B, const u32 (&off)[4], uint64_t *okeys,
                                            uint32_t *oids, uint64_t out_cap, uint64_t *pk,
                                            uint64_t pk_cap) {
#pragma unroll
    for (u32 p = 0; p < 4; p++) {
        if (p >= B.npass) break; /* wave-uniform */
        if (!B.ok[p]) continue;
        const u32 j = B.jb[p];
        const u64 o = (u64)(j == 0 ? off[0] : j == 1 ? off[1] : j == 2 ? off[2] : off[3]) + B.r;
        if (o < out_cap) {
            okeys[o] = B.k[p];
            oids[o] = B.id[p];
        }
        if (pk && o < pk_cap) {
            pk[1 + o] = B.k[p];
            ((uint32_t *)(pk + 1 + pk_cap))[o] = B.id[p];
        }
    }
}

/* any lane's c: one v_cmp into a scalar mask and a scalar test (__any's
 * lowering re-materialized the mask as a lane value and compared again) */
__device__ __forceinline__ bool wave_any(bool c) { return __builtin_amdgcn_ballot_w64(c) != 0; }

/* wave-wide exclusive prefix sum of a small per-lane count */
__device__ __forceinline__ u32 wave_excl_scan(u32 v, u32 *total) {
    u32 lane = lane_id();
    u32 x = v;
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        u32 y = shfl_up_u32(x, d);
        if (lane >= (u32)d) x += y;
    }
    *total = shfl_u32(x, WAVE - 1);
    return x - v;
}

/* A byte of A inside [lo, hi) when `want`, else 0.  Branch-free: the load
 * always issues, from `safe` (any valid device byte) when the byte is not
 * wanted, so several of these go out together -- as guarded loads, each
 * in its own EXEC-masked block, the compiler waited for one before issuing
 * the next (a segment start took 4 serial round trips for 4 bytes). */
__device__ __forceinline__ u8 load_byte_masked(const u8 *A, int64_t aoff, int64_t lo, int64_t hi,
                                               bool want, const u8 *safe) {
    const bool ok = want && aoff >= lo && aoff < hi;
    typedef const __attribute__((address_space(1))) u8 gu8;
    const u8 v = *(gu8 *)(ok ? A + aoff : safe);
    return ok ? v : (u8)0;
}

/* A segment's block record (i wave-uniform), read as scalar loads: the
 * table is written by the host before the launch and only read here.  As
 * vector loads the record went through the few VGPRs free at a segment
 * start, one load waited for before the next -- four serial round trips
 * per segment; scalar loads all go out at once. */
__device__ __forceinline__ VsaBlock load_block(const VsaBlock *blocks, u32 i) {
    static_assert(sizeof(VsaBlock) == 9 * sizeof(u64), "VsaBlock: 9 words");
    typedef const __attribute__((address_space(4))) u64 cu64;
    cu64 *p = (cu64 *)(blocks + i);
    u64 w[9];
#pragma unroll
    for (int k = 0; k < 9; k++) w[k] = p[k];
    VsaBlock b;
    __builtin_memcpy(&b, w, sizeof(b));
    return b;
}

/* ===================================================== literal scan === */

template <int MODE>
struct LitTraits;

/* Teddy: the first stage is an exact per-byte table derived from the
 * confirm records (runtime.hip derive_teddy_table), 8 positions x 8
 * buckets; the reference's nibble masks (teddy_compile.cpp:439) admit up to
 * 36 byte pairs per bucket and position where the literals have 6 */
template <>
struct LitTraits<VSA_MODE_TEDDY> {
    static constexpr int LB = 8;
    /* 4 of the table's 8 positions (its low dword): a byte of each of the
     * last 4 literal bytes, exact, passes ~48 / 95^4 of random positions at
     * cfg 3 -- the u64 entries' other 4 fields bought no candidates worth
     * their accumulate (39 VALU against 22 for u32 entries, fdr4_acc_*) */
    static constexpr int NL = 4;
    static constexpr int CW = 4;
    static constexpr int EW = 3;
    typedef u32 S_t;
};
template <>
struct LitTraits<VSA_MODE_NOOD> {
    static constexpr int LB = 8;
    static constexpr int NL = 1; /* no look-back state */
    static constexpr int CW = 1;
    static constexpr int EW = 2; /* {meta}, {hits} */
    typedef u32 S_t;
};
template <>
struct LitTraits<VSA_MODE_FAT> {
    static constexpr int LB = 16;
    static constexpr int NL = 4;
    static constexpr int CW = 8;
    static constexpr int EW = 4;
    typedef u64 S_t;
};
/* FDR engines, 4-field first stage (runtime.hip derive_fdr4_table): u32
 * entries, 4 ends x 8 buckets, keyed by 15 bits of the 3 bytes ending at
 * the position (vsa_fdr4_key) */
template <>
struct LitTraits<VSA_MODE_FDR4> {
    static constexpr int LB = 8;
    static constexpr int NL = 4;
    static constexpr int CW = 4;
    static constexpr int EW = 3;
    typedef u32 S_t;
};

/* per-bucket confirm parameters staged in LDS (FDRConfirm, fdr_confirm.h:78) */
struct PfRec {
    u64 andmsk;
    u32 slot_off; /* word offset of the bucket's slot bitmap, ~0 = none */
    u32 shift;    /* 64 - nBits */
};

struct ConfLds {
    u64 andmsk[16];
    u64 mult[16];
    u32 nbits[16];
    u32 off[16];
    PfRec pf[16]; /* one 32-B record per bucket for the scanners' prefilter */
    /* the sort bins this workgroup owns alone, [lb_lo, lb_lo + lb_n)
     * (runtime.hip plan_wg_bins): their record counts, kept here and
     * stored to bin_counts when the confirm waves are done */
    u32 lb_lo, lb_n;
    u32 lbins[VSA_LBINS];
    u32 nrec; /* binned sort: records confirmed here (one global add at the end) */
    /* fused finish: the local bins cover ends [f_lo, f_lo + lb_n << f_shift)
     * (lb_lo = 0) */
    u64 f_lo;
    u32 f_shift;
    u32 f_bad;  /* a record outside the local bins (a crowd for the host) */
    u32 f_cand; /* counters[2]'s part from this workgroup (the publisher sums) */
};

/* a record's sort bin: the end's global bin, or under the fused finish its
 * local bin (end - f_lo) >> f_shift, whose staging row is the workgroup's
 * own (bin_row) */
__device__ __forceinline__ u32 rec_bin(const VsaLitParams &P, const ConfLds &cl, u64 end) {
    if (P.fin_keys) {
        const u64 d = (end - cl.f_lo) >> cl.f_shift; /* an end below f_lo wraps: out of range */
        return d < VSA_LBINS ? (u32)d : 0xffffffffu;
    }
    return (u32)(end >> P.bin_shift);
}
__device__ __forceinline__ size_t bin_row(const VsaLitParams &P, u32 bin) {
    return P.fin_keys ? (size_t)blockIdx.x * VSA_LBINS + bin : (size_t)bin;
}

/* a record's slot in its sort bin: an owned bin's from the workgroup's LDS
 * count (no global round trip), any other bin's from the global one.  Under
 * the fused finish every record's bin is local; one outside the local range
 * (the plan guarantees none) counts as a crowd, so the host rescans */
__device__ __forceinline__ u32 bin_slot_take(const VsaLitParams &P, const ConfLds &cl, u32 bin) {
    const u32 k = bin - cl.lb_lo;
    if (k < cl.lb_n)
        return __hip_atomic_fetch_add(const_cast<u32 *>(&cl.lbins[k]), 1u, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
    if (P.fin_keys) {
        __hip_atomic_store(const_cast<u32 *>(&cl.f_bad), 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
        return VSA_SORT_BIN_MAX;
    }
    return __hip_atomic_fetch_add(&P.bin_counts[bin], 1u, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
}

/* counters[VSA_CTR_BIN_OVERFLOW] = 1 as an agent-scope atomic store: the
 * fused finish's last workgroup reads it from another XCD */
__device__ __forceinline__ void flag_crowd(const VsaLitParams &P) {
    __hip_atomic_store(&P.counters[VSA_CTR_BIN_OVERFLOW], 1ULL, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

/* confirm-queue entry (the confirm wave's private queue): meta = aoff << 24 |
 * blk << 4 | bucket; key = 8 bytes ending at the candidate end (bytes
 * before the block are 0, fdr.c:798-806) */
struct QEnt {
    u64 meta;
    u64 key;
};

/* Candidates go from the scanning waves to the workgroup's confirm wave
 * through per-wave single-producer LDS rings of 2^lg chunk entries: one
 * entry per lane whose 16 ends hold any first-stage candidate, carrying the
 * lane's candidate masks and the 24 bytes its confirm keys are cut from, so
 * the scanning wave never loops over candidate bits (the confirm wave
 * expands the entries 64 at a time).  Entry layout, EW uint4 words: {meta,
 * c[0..CW), pv2, pv3, d0..d3} (noodle: {meta}, {hits}), meta = p0 | blk << 40.  A scanning wave owns its ring's head (a register: no atomic,
 * no LDS round trip on a push), waits for room only against its cached
 * copy of the tail the confirm wave publishes, writes the entries and then
 * publishes its head with a plain LDS store (LDS executes a wave's
 * instructions in order, so a visible head implies visible entries).  The
 * confirm wave polls the 15 heads with one broadcast read (lane 4 r + k
 * reads head r) and then reads only the available slots tail_r + k, k < 4:
 * one instruction per idle poll, and masked lanes cost no LDS banks.  (A
 * shared ring reserved with a returning LDS atomic cost the scanners that
 * atomic's round trip on every push, ~1000 cycles under the bank-conflicted
 * lookups.) */
#define ENT_BLK_SHIFT 40
#define ENT_LAP_SHIFT 60
#define ENT_P0_MASK ((1ULL << ENT_BLK_SHIFT) - 1)
struct LitShared {
    const void *tab;
    u32 tab_lds;     /* LDS byte address of tab (LDS tables) */
    u32 tsel;        /* Teddy: TEDDY_TAB_LDS | this lane's copy offset */
    uint4 *ring;     /* this wave's ring */
    const u32 *tail; /* this ring's consumed position (written by the confirm wave) */
    u32 *head;       /* this ring's published head (written by this wave) */
    u32 lg;          /* log2 ring entries (>= 2) */
    u32 dbg;         /* VsaLitParams.dbg */
    const u32 *slots; /* slot bitmaps (LDS; scanner expansion, XP) */
    unsigned long long *diag; /* LDS: candidate-path cycles (dbg & 32768) */
};

__device__ __forceinline__ u32 lds_ld32(const u32 *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st32(u32 *p, u32 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ u32 conf_hash(u64 key, u64 andmsk, u64 mult, u32 nbits) {
    return (u32)(((key & andmsk) * mult) >> (64 - nbits));
}

/* Exact confirm of up to CU candidates per lane (fdr_confirm_runtime.h:43-102
 * minus the sequential state, which the host replays): for each, walk the
 * LitInfo chain of litIndex[hash] and emit every literal with (key & msk) ==
 * v whose start lies inside the block.  The candidates' global loads
 * (litIndex slot, block record, each chain step) are independent, so they
 * are issued together: one memory latency per chain step for all of them. */
template <int CONF_U>
__device__ __forceinline__ void confirm_multi(const VsaLitParams &P, const ConfLds &cl,
                                              const QEnt (&q)[CONF_U], const bool (&valid)[CONF_U],
                                              u32 mis) {
    /* LitInfo addresses as u32 offsets from confBase (an SGPR base: one
     * VGPR per candidate instead of two) */
    u32 fc[CONF_U], li[CONF_U];
    u32 st[CONF_U], b[CONF_U];
    u64 base[CONF_U], blen[CONF_U];
    int64_t hlen[CONF_U], e[CONF_U];
#pragma unroll
    for (int i = 0; i < CONF_U; i++) {
        b[i] = (u32)(q[i].meta & 15);
        const u32 blk = (u32)((q[i].meta >> 4) & 0xfffff);
        fc[i] = cl.off[b[i]];
        st[i] = 0;
        base[i] = 0;
        blen[i] = ~0ULL;
        hlen[i] = 0;
        if (valid[i]) {
            const u32 c = conf_hash(q[i].key, cl.andmsk[b[i]], cl.mult[b[i]], cl.nbits[b[i]]);
            st[i] = *((const u32 *)(P.conf_base + fc[i] + 32) + c);
            base[i] = P.blocks[blk].base;
            blen[i] = P.blocks[blk].len;
            hlen[i] = (int64_t)P.blocks[blk].hlen;
        }
    }
    bool live[CONF_U];
#pragma unroll
    for (int i = 0; i < CONF_U; i++) {
        live[i] = st[i] != 0;
        li[i] = fc[i] + st[i];
        e[i] = (int64_t)((q[i].meta >> 24) - mis - base[i]); /* block-relative end */
        /* runs (VSA_BLK_RUN): an end past the entry's block is in the next,
         * back-to-back block (>= 1 KiB: at most one boundary per chunk);
         * outside runs every end lies inside its block */
        if (e[i] >= (int64_t)blen[i]) {
            const VsaBlock &nb = P.blocks[((q[i].meta >> 4) & 0xfffff) + 1];
            base[i] += blen[i];
            e[i] -= (int64_t)blen[i];
            hlen[i] = (int64_t)nb.hlen;
        }
    }
    /* wave-uniform loop (every lane stays in, so the output slot reservation
     * below is one atomic per wave and step, not one per match: a single
     * returning atomic word saturates near 90 per microsecond chip-wide) */
    for (;;) {
        bool any = false;
#pragma unroll
        for (int i = 0; i < CONF_U; i++) any |= live[i];
        if (!__any(any)) break;
        uint4 w0[CONF_U], w1[CONF_U];
#pragma unroll
        for (int i = 0; i < CONF_U; i++) {
            if (live[i]) {
                w0[i] = *(const uint4 *)(P.conf_base + li[i]);        /* v, msk */
                w1[i] = *(const uint4 *)(P.conf_base + li[i] + 16); /* groups | id,size,flags,next */
            }
        }
        bool mt[CONF_U];
        u64 pm[CONF_U]; /* wave-uniform */
        u32 tot = 0;
#pragma unroll
        for (int i = 0; i < CONF_U; i++) {
            mt[i] = false;
            if (live[i]) {
                const u64 v = ((u64)w0[i].y << 32) | w0[i].x;
                const u64 msk = ((u64)w0[i].w << 32) | w0[i].z;
                const u32 size = w1[i].w & 0xff;
                mt[i] = (q[i].key & msk) == v && e[i] + 1 + hlen[i] >= (int64_t)size;
            }
            pm[i] = __ballot(mt[i]);
            tot += (u32)__popcll(pm[i]);
        }
        if (tot) {
            /* binned sort on: each match goes straight into its sort bin (an
             * owned bin's slot from LDS, others' from a returning atomic)
             * and is counted in LDS (cl.nrec, added to counters[0] once per
             * workgroup): a confirm step neither waits on an output
             * reservation nor adds to the one word every workgroup shares
             * (profiles/r05/r05zl_bin_records_ab.txt).  Off: output slots
             * from one returning atomic per wave and step */
            const bool bins = P.bin_keys != nullptr;
            unsigned long long s0 = 0;
            if (lane_id() == 0) {
                if (bins)
                    __hip_atomic_fetch_add(const_cast<u32 *>(&cl.nrec), tot, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                else
                    s0 = atomicAdd(&P.counters[0], (unsigned long long)tot);
            }
            const u64 sb = ((u64)readlane_u32((u32)(s0 >> 32), 0) << 32) | readlane_u32((u32)s0, 0);
            u32 bslot[CONF_U], bbin[CONF_U];
#pragma unroll
            for (int i = 0; i < CONF_U; i++)
                if (bins && mt[i]) {
                    bbin[i] = rec_bin(P, cl, base[i] + (u64)e[i]);
                    bslot[i] = bin_slot_take(P, cl, bbin[i]);
                }
#pragma unroll
            for (int i = 0; i < CONF_U; i++) {
                if (!mt[i]) continue;
                const u64 end = base[i] + (u64)e[i];
                const u64 lidx = (u64)((li[i] - fc[i]) >> 3) & VSA_KEY_LI_MASK;
                u32 before = 0; /* this lane's rank among the step's matches */
#pragma unroll
                for (int k = 0; k < i; k++) before += (u32)__popcll(pm[k]);
                const u64 q = bins ? (u64)bin_row(P, bbin[i]) * VSA_SORT_BIN_MAX + bslot[i]
                                   : sb + before + __builtin_amdgcn_mbcnt_hi(
                                         (u32)(pm[i] >> 32), __builtin_amdgcn_mbcnt_lo((u32)pm[i], 0));
                if (bins ? bslot[i] < VSA_SORT_BIN_MAX : q < P.out_cap) {
                    (bins ? P.bin_keys : P.out_keys)[q] = (end << VSA_KEY_END_SHIFT) |
                                                          ((u64)b[i] << VSA_KEY_BUCKET_SHIFT) | lidx;
                    (bins ? P.bin_ids : P.out_ids)[q] = w1[i].z;
                } else if (bins) {
                    flag_crowd(P); /* crowded: the host rescans without bins */
                }
            }
        }
#pragma unroll
        for (int i = 0; i < CONF_U; i++) {
            if (!live[i]) continue;
            li[i] += 32;
            live[i] = ((w1[i].w >> 16) & 0xff) != 0;
        }
    }
}

template <int MODE>
__device__ __forceinline__ u64 lit_lookup(const void *tab, u32 key, u32 lane) {
    if constexpr (MODE == VSA_MODE_FDR4) {
        (void)lane;
        return ((const u32 *)tab)[key];
    } else if constexpr (MODE == VSA_MODE_TEDDY) {
        /* u32 rows of 256 B: the lane's copy at (lane & 31) * 4 */
        return ((const u32 *)tab)[(key << 6) | (lane & 31)];
    } else {
        return ((const u64 *)tab)[(key << 5) | (lane & 31)];
    }
}

struct IterState {
    u64 carry;  /* pending table contributions into the next chunk's first ends */
    u64 pbytes; /* the 8 bytes before the next chunk (lane 63's d[2..3]) */
    /* FDR4 sweep: lane 0 holds the previous chunk's lane-63 d[3] / U[4]
     * (lane_ror1 of them); carry and pbytes' high half are refreshed from
     * these only when the sweep ends (sweep_enter / sweep_leave) */
    u32 p3, p4;
    u32 ncand;  /* first-stage candidates so far (diagnostic, wave-uniform) */
    u32 tail_cache; /* last tail read from the confirm wave */
    u32 head;       /* entries this wave has pushed to its ring */
    /* scanner expansion (xp_push): a batch of expanded candidates, one per
     * lane in lanes [0, xn) -- match key (qm) and 8-byte confirm key --
     * prefiltered and pushed together once 64 have gathered (xp_flush) */
    u32 xs[4];
    u32 xn;
};

struct SegCtx {
    u32 blk;
    int64_t blo, bhi; /* aoff of the block */
    int64_t vlo;      /* lowest readable aoff (blo - history) */
    int64_t start, len, zbase;
    int64_t rlo;      /* lowest reported end: max(start, block rlo) */
    int64_t qlo;      /* Teddy: lowest looked-up position (block-relative) */
    int64_t run_nxt;  /* runs: aoff where block blk + 1 starts (else INT64_MAX) */
    bool stream;      /* streaming with history: no FDR start state */
};

/* Append one EW-word entry per lane with push set to the wave's ring
 * (wave-uniform call), in batches of at most the ring size.  The head and
 * tail cache in `st` are updated identically by every lane. */
template <int EW, typename ST>
__device__ __forceinline__ void ring_push(const LitShared &L, ST &st, bool push,
                                          const u32 (&w)[4 * EW]) {
    const u64 pm = __ballot(push);
    if (pm == 0) return;
    const u32 n = (u32)__popcll(pm);
    const u32 r = __builtin_amdgcn_mbcnt_hi((u32)(pm >> 32),
                                             __builtin_amdgcn_mbcnt_lo((u32)pm, 0));
    const u32 cap = 1u << L.lg;
    for (u32 b0 = 0; b0 < n; b0 += cap) {
        const u32 m = n - b0 < cap ? n - b0 : cap;
        const u32 pos = st.head;
        if (pos + m - st.tail_cache > cap) {
            for (;;) {
                st.tail_cache = readfirstlane_u32(lds_ld32(L.tail));
                if (pos + m - st.tail_cache <= cap) break;
                __builtin_amdgcn_s_sleep(2);
            }
        }
        if (push && r >= b0 && r < b0 + m) {
            const u32 slot = pos + r - b0;
            uint4 *q = L.ring + (size_t)(slot & (cap - 1)) * EW;
#pragma unroll
            for (int k = 0; k < EW; k++)
                if (k < 2 || !VSA_DBG(L.dbg, 256)) /* experiment: short entries */
                    q[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
        }
        st.head = pos + m;
        /* the batch's entries before its head (a later batch may wait for
         * the confirm wave to drain this one) */
        asm volatile("" ::: "memory");
        if (lane_id() == 0) lds_st32(L.head, st.head);
    }
}

/* Shift-or of one lane's 16 table entries (the reference's running state,
 * fdr.c:145-296 / teddy.c:921-971, restated without a serial chain): field
 * k (LB bits) of x[j] is OR-ed into the conf field of end j + k.  Entries
 * are grouped by j mod (32 / LB) so each group ORs dword-aligned, and each
 * group is then shifted into place once (alignbyte) — 39 VALU for FDR's 16
 * u64 entries against 64 for a per-position shift.  c = the conf fields of
 * the lane's own 16 ends, s_out = the fields spilling into ends 16.. */
__device__ __forceinline__ void fdr4_acc_even(const u32 (&x)[16], u32 (&U)[5]);
__device__ __forceinline__ void fdr4_acc_odd(const u32 (&x)[16], u32 (&U)[5]);
template <int MODE>
__device__ __forceinline__ void conf_accumulate(const typename LitTraits<MODE>::S_t (&x)[16],
                                                u32 (&c)[LitTraits<MODE>::CW], u64 &s_out) {
    auto lo = [&](int j) { return (u32)(u64)x[j]; };
    auto hi = [&](int j) { return (u32)((u64)x[j] >> 32); };
    if constexpr (MODE == VSA_MODE_TEDDY) {
        /* u32 entries, 4 fields: FDR4's OR-into-place (field f of x[p] onto
         * end p + f; U[4] = ends 16..18, the next lane's 0..2) */
        u32 U[5];
        fdr4_acc_even(x, U);
        fdr4_acc_odd(x, U);
#pragma unroll
        for (int i = 0; i < 4; i++) c[i] = U[i];
        s_out = U[4];
    } else if constexpr (LitTraits<MODE>::LB == 8) {
        /* A[r][w] = dword w of the group j = 4 w' + r (before its r-byte
         * shift); group 0 is folded straight into F */
        u32 A[4][5];
#pragma unroll
        for (int r = 1; r < 4; r++) {
            A[r][0] = lo(r);
            A[r][1] = hi(r) | lo(4 + r);
            A[r][2] = hi(4 + r) | lo(8 + r);
            A[r][3] = hi(8 + r) | lo(12 + r);
            A[r][4] = hi(12 + r);
        }
        u32 F[6];
        F[0] = lo(0) | (A[1][0] << 8) | (A[2][0] << 16) | (A[3][0] << 24);
#pragma unroll
        for (int i = 1; i < 5; i++) {
            const u32 g0a = hi(4 * (i - 1));
            const u32 g0b = i < 4 ? lo(4 * i) : 0u;
            const u32 s1 = __builtin_amdgcn_alignbyte(A[1][i], A[1][i - 1], 3);
            const u32 s2 = __builtin_amdgcn_alignbyte(A[2][i], A[2][i - 1], 2);
            const u32 s3 = __builtin_amdgcn_alignbyte(A[3][i], A[3][i - 1], 1);
            F[i] = or3(or3(g0a, g0b, s1), s2, s3);
        }
        F[5] = or3(A[1][4] >> 24, A[2][4] >> 16, A[3][4] >> 8);
#pragma unroll
        for (int i = 0; i < 4; i++) c[i] = F[i];
        s_out = ((u64)F[5] << 32) | F[4];
    } else {
        /* 16-bit fields: even j land dword-aligned, odd j half a dword up */
        u32 A0[9], A1[9];
        A0[0] = lo(0);
        A1[0] = lo(1);
#pragma unroll
        for (int w = 1; w < 8; w++) {
            A0[w] = hi(2 * w - 2) | lo(2 * w);
            A1[w] = hi(2 * w - 1) | lo(2 * w + 1);
        }
        A0[8] = hi(14);
        A1[8] = hi(15);
        u32 F[10];
        F[0] = A0[0] | (A1[0] << 16);
#pragma unroll
        for (int i = 1; i < 9; i++) F[i] = A0[i] | __builtin_amdgcn_alignbyte(A1[i], A1[i - 1], 2);
        F[9] = A1[8] >> 16;
#pragma unroll
        for (int i = 0; i < 8; i++) c[i] = F[i];
        s_out = ((u64)F[9] << 32) | F[8];
    }
}

/* ---- FDR4: the 4-field first stage (VSA_MODE_FDR4) ----
 * Lane l looks up positions 0 .. 15 of its chunk; the key of position p is
 * vsa_fdr4_key(b[p-2], b[p-1], b[p]) (bytes -2, -1: the previous lane's, or
 * chunk's, last ones) and field f (byte f) of the entry applies to end p + f.
 * U[0..3] = the conf bytes of ends 0 .. 15, U[4] bytes 0..2 = ends 16..18,
 * which are the next lane's ends 0..2 (spilled once per iteration).
 *
 * Keys, two per dword, one per 16-bit half: [b[p-1] & 0x7f | (b[p-2] & 1)
 * << 7, b[p] & 0x7f] (vsa_fdr4_key's bit order: the halves of the 7-bit
 * bytes as they lie in memory, with bit 0 of the byte before them in the
 * first byte's free bit 7).  From z = the chunk's bytes & 0x7f: the even
 * positions (4w, 4w + 2) take t = bytes 4w-1 .. 4w+2 (v_alignbyte) and the
 * odd ones (4w + 1, 4w + 3) z[w] itself; the b[p-2] bits come by one
 * funnel shift (v_alignbit) and one v_bfi each.  Six VALU ops per four keys
 * (nine with the round-3 key order, which shifted each half by one). */
__device__ __forceinline__ u32 bfi_b32(u32 m, u32 a, u32 b) {
    u32 r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(m), "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ void fdr4_keys(const u32 (&d)[4], u32 pv3, u32 (&ke)[4],
                                          u32 (&ko)[4]) {
    /* the byte mask kept in a VGPR: v_and_b32 with two VGPR operands issues
     * in half the cycles of one with a constant (tools/probe_issue.hip) */
    u32 m7;
    asm("v_mov_b32 %0, 0x7f7f7f7f" : "=v"(m7));
    u32 z[4];
#pragma unroll
    for (int w = 0; w < 4; w++) asm("v_and_b32 %0, %1, %2" : "=v"(z[w]) : "v"(m7), "v"(d[w]));
    u32 zp;
    asm("v_and_b32 %0, %1, %2" : "=v"(zp) : "v"(m7), "v"(pv3));
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const u32 zq = w ? z[w - 1] : zp;
        /* bit 7 = bit 0 of b(4w-2), bit 23 = of b(4w) (even); b(4w-1),
         * b(4w+1) (odd) */
        ke[w] = bfi_b32(0x00800080u, __builtin_amdgcn_alignbit(z[w], zq, 9),
                        __builtin_amdgcn_alignbyte(z[w], zq, 3));
        ko[w] = bfi_b32(0x00800080u, __builtin_amdgcn_alignbit(z[w], zq, 17), z[w]);
    }
}
/* LDS byte address of a u32 entry: base + 4 * (16-bit half H of w) */
template <int H>
__device__ __forceinline__ u32 tab_addr16x4(u32 w, u32 base) {
    u32 r;
    if constexpr (H == 0)
        asm("v_mad_u32_u16 %0, %1, 4, %2" : "=v"(r) : "v"(w), "s"(base));
    else
        asm("v_mad_u32_u16 %0, %1, 4, %2 op_sel:[1,0,0,0]" : "=v"(r) : "v"(w), "s"(base));
    return r;
}
__device__ __forceinline__ u32 lds_ld32a(u32 addr) {
    return *(const __attribute__((address_space(3))) u32 *)(uintptr_t)addr;
}
/* Two LDS reads in the lanes of m only (EXEC = m around them; a lane
 * outside m keeps whatever its registers held, which only ever reaches ends
 * that are already dead).  The compiler does not see these reads: the
 * caller waits for them (lds_wait8) before the values are used.  Reads the
 * compiler issued are counted with them, so its own waits stay correct, if
 * conservative. */
__device__ __forceinline__ void lds_ld32x2_masked(u64 m, u32 a0, u32 a1, u32 &x0, u32 &x1) {
    u64 sv;
    asm volatile("s_mov_b64 %2, exec\n\t"
                 "s_mov_b64 exec, %5\n\t"
                 "ds_read_b32 %0, %3\n\t"
                 "ds_read_b32 %1, %4\n\t"
                 "s_mov_b64 exec, %2"
                 : "=&v"(x0), "=&v"(x1), "=&s"(sv)
                 : "v"(a0), "v"(a1), "s"(m));
}
__device__ __forceinline__ void lds_wait8(u32 (&x)[16]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(x[1]), "+v"(x[3]), "+v"(x[5]), "+v"(x[7]), "+v"(x[9]), "+v"(x[11]),
                   "+v"(x[13]), "+v"(x[15]));
}
/* OR-into-place: field f of x[p] onto end p + f.  EVEN: x[0, 2, .., 14]
 * (the first writes of U); ODD: x[1, 3, .., 15] OR-ed on top. */
__device__ __forceinline__ void fdr4_acc_even(const u32 (&x)[16], u32 (&U)[5]) {
    U[0] = x[0] | (x[2] << 16);
#pragma unroll
    for (int k = 1; k < 4; k++) U[k] = x[4 * k] | __builtin_amdgcn_alignbyte(x[4 * k + 2], x[4 * k - 2], 2);
    U[4] = x[14] >> 16;
}
__device__ __forceinline__ void fdr4_acc_odd(const u32 (&x)[16], u32 (&U)[5]) {
    U[0] = or3(U[0], x[1] << 8, x[3] << 24);
#pragma unroll
    for (int k = 1; k < 4; k++)
        U[k] = or3(U[k], __builtin_amdgcn_alignbyte(x[4 * k + 1], x[4 * k - 3], 3),
                   __builtin_amdgcn_alignbyte(x[4 * k + 3], x[4 * k - 1], 1));
    U[4] = or3(U[4], x[13] >> 24, x[15] >> 8);
}
/* One chunk's conf bytes (before the previous lane's spill into U[0]).
 * Sweep (LOOKM == false): two levels -- the even positions for every lane,
 * then the odd ones only in lanes where a conf dword they reach is still
 * live (EXEC-masked reads: a lane left out takes no LDS bank and no VALU
 * op; its stale value is OR-ed only into ends already dead, so the result
 * is the one-level filter's).  Edge iterations (LOOKM): one level, position
 * p looked up only where bit p of look_m is set. */
template <bool LOOKM>
__device__ __forceinline__ void fdr4_conf(const LitShared &L, const u32 (&d)[4], u32 pv3,
                                          u32 look_m, u32 (&U)[5]) {
    u32 ke[4], ko[4], x[16];
    fdr4_keys(d, pv3, ke, ko);
    auto ld = [&](int p, u32 a) {
        if (LOOKM) x[p] = ((look_m >> p) & 1u) ? lds_ld32a(a) : 0u;
        else x[p] = lds_ld32a(a);
    };
#pragma unroll
    for (int w = 0; w < 4; w++) {
        ld(4 * w, tab_addr16x4<0>(ke[w], L.tab_lds));
        ld(4 * w + 2, tab_addr16x4<1>(ke[w], L.tab_lds));
    }
    if (LOOKM) {
#pragma unroll
        for (int w = 0; w < 4; w++) {
            ld(4 * w + 1, tab_addr16x4<0>(ko[w], L.tab_lds));
            ld(4 * w + 3, tab_addr16x4<1>(ko[w], L.tab_lds));
        }
        fdr4_acc_even(x, U);
        fdr4_acc_odd(x, U);
        return;
    }
    fdr4_acc_even(x, U);
    /* odd key dword w (positions 4w + 1, 4w + 3) reaches ends 4w + 1 ..
     * 4w + 6: gated on conf dwords w and w + 1 (lanes with one live end
     * among 4w .. 4w + 7; 28 % of them on cfg-4 text).  One gate per slot
     * (exact 4 ends: 15 % real lookups) measured slower -- 0.985 against
     * 0.919 ms: its 20 more VALU per iteration cost more than the LDS
     * conflicts it saves (profiles/r03_fdr4_gate_ab.txt). */
    u64 m[5];
#pragma unroll
    for (int k = 0; k < 4; k++) m[k] = __builtin_amdgcn_ballot_w64(U[k] != 0xffffffffu);
    /* ends 16..18 are the next lane's ends 0..2: live unless that lane's own
     * level 1 already killed its ends 0..3 (bit l + 1 of m[0]; lane 63's next
     * lane is the next chunk's lane 0, unknown here, so live).  U[4] itself
     * always has end 18 live: level 1 never reaches it. */
    m[4] = (m[0] >> 1) | (1ull << 63);
#pragma unroll
    for (int w = 0; w < 4; w++)
        lds_ld32x2_masked(m[w] | m[w + 1], tab_addr16x4<0>(ko[w], L.tab_lds),
                          tab_addr16x4<1>(ko[w], L.tab_lds), x[4 * w + 1], x[4 * w + 3]);
    lds_wait8(x);
    fdr4_acc_odd(x, U);
}

/* Block-edge masks: position j (0..16) of a lane's chunk is end / byte
 * q0 + j (block-relative).  rel32 clamps a bound X to the chunk's
 * coordinates; range_mask gives bits j in [lo, hi) over 17 positions, so an
 * edge iteration's per-position tests are a handful of 32-bit ops instead
 * of 16 x 64-bit compares each. */
__device__ __forceinline__ int rel32(int64_t x, int64_t q0) {
    const int64_t d = x - q0;
    return d < -1 ? -1 : (d > 17 ? 17 : (int)d);
}
__device__ __forceinline__ u32 range_mask(int lo, int hi) {
    lo = lo < 0 ? 0 : lo;
    hi = hi > 17 ? 17 : hi;
    return hi <= lo ? 0u : ((0xffffffffu << lo) & ((1u << hi) - 1u));
}
/* bits 0..3 of t -> bytes 0..3 of 0xff / 0 (no carries: the shifted copies
 * of t do not overlap) */
__device__ __forceinline__ u32 nib_to_bytes(u32 t) {
    return (((t & 0xfu) * 0x00204081u) & 0x01010101u) * 0xffu;
}
/* 4 bytes at signed byte offset o of the zero-padded 16-byte s[0..3] */
__device__ __forceinline__ u32 window4(const u32 (&s)[4], int o) {
    const int a = o >> 2; /* floor */
    const u32 b = (u32)o & 3u;
    auto W = [&](int i) -> u32 {
        u32 v = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) v = i == k ? s[k] : v;
        return v;
    };
    return __builtin_amdgcn_alignbyte(W(a + 1), W(a), b);
}

/* Scanner expansion (XP, large literal sets): the scanning wave expands its
 * candidate bits itself and pushes only the ones the bucket's slot bitmap
 * passes (litIndex[hash] == 0 rejects, fdr_confirm_runtime.h:43-60), as
 * confirm-queue entries (QEnt), to its ring; the confirm wave only
 * confirms.  With thousands of literals per bucket the first stage passes
 * ~1e-2 candidate bits per byte (20k literals: ~9 per 1 KiB iteration, in
 * ~1.5 rounds of one bit per lane).
 * Round 4: the rounds only extract -- each round every lane takes its
 * lowest remaining (end, bucket) bit and cuts its 8-byte key from the bytes
 * it holds (branch-free) -- and one ds_permute per word packs the round's
 * bits into consecutive lanes of a batch (IterState xs / xn) that outlives
 * the iteration; the prefilter (bucket record, hash, slot word: two
 * dependent LDS reads) and the ring push run once per 64 candidates
 * (xp_flush) instead of once per round with a few lanes busy.
 * c = candidate bits of ends 0..15 (byte i of c[w] = end 4 w + i, bit =
 * bucket); meta = p0 | blk << ENT_BLK_SHIFT; D = bytes p0 - 8 .. p0 + 15. */
template <typename ST>
__device__ __forceinline__ void xp_flush(const VsaLitParams &P, const ConfLds &cl,
                                         const LitShared &L, ST &st) {
    const u32 n = st.xn;
    if (n == 0) return;
    const bool act = lane_id() < n;
    const u64 key = ((u64)st.xs[3] << 32) | st.xs[2];
    const u32 bb = st.xs[0] & 7u;
    const PfRec pf = cl.pf[bb];
    const bool chk = act && pf.slot_off != 0xffffffffu;
    const u32 h = (u32)(((key & pf.andmsk) * P.pf_mult) >> pf.shift);
    const u32 sw = chk ? lds_ld32(&L.slots[pf.slot_off + (h >> 5)]) : ~0u;
    const bool push = act && ((sw >> (h & 31)) & 1u);
    const u32 w[4] = {st.xs[0], st.xs[1], st.xs[2], st.xs[3]};
    ring_push<1>(L, st, push, w);
    st.xn = 0;
}

__device__ __forceinline__ void xp_push(const VsaLitParams &P, const ConfLds &cl,
                                        const LitShared &L, IterState &st, u32 (&c)[4],
                                        u64 meta, u32 pv2, u32 pv3, const u32 (&d)[4]) {
    const u32 D[6] = {pv2, pv3, d[0], d[1], d[2], d[3]};
    const u64 p0 = meta & ENT_P0_MASK;
    const u64 blk4 = (meta >> ENT_BLK_SHIFT) << 4;
    const u32 lane = lane_id();
    /* the 128 candidate bits as two 64-bit halves: bit b is end b >> 3,
     * bucket b & 7 (byte i of c[w] = end 4 w + i), so a round's lowest bit
     * is one 64-bit find-first and its clear one 64-bit a & (a - 1), with no
     * per-word select */
    u64 lo = ((u64)c[1] << 32) | c[0];
    u64 hi = ((u64)c[3] << 32) | c[2];
    for (;;) {
        const bool have = (lo | hi) != 0;
        const u64 B = __ballot(have);
        if (B == 0) break;
        const u32 cnt = (u32)__popcll(B);
        if (st.xn + cnt > WAVE) xp_flush(P, cl, L, st);
        const bool inlo = lo != 0;
        const u64 cur = inlo ? lo : hi;
        const u32 b = (inlo ? 0u : 64u) + (u32)__builtin_ctzll(cur | (1ull << 63));
        const u64 nxt = cur & (cur - 1);
        lo = inlo ? nxt : lo;
        hi = inlo ? hi : nxt;
        const u32 jj = b >> 3, bb = b & 7;
        /* key = bytes [jj - 7, jj] = byte offset o = jj + 1 .. jj + 8 of D:
         * dwords a, a + 1, a + 2 shifted by o & 3 */
        const u32 o = jj + 1, a = o >> 2, sh = o & 3u;
        u32 x0 = D[0], x1 = D[1], x2 = D[2];
#pragma unroll
        for (int k = 1; k < 5; k++) {
            const bool sel = a == (u32)k;
            x0 = sel ? D[k] : x0;
            x1 = sel ? D[k + 1] : x1;
            x2 = sel ? D[k + 2 < 6 ? k + 2 : 5] : x2;
        }
        const u32 key_lo = __builtin_amdgcn_alignbyte(x1, x0, sh);
        const u32 key_hi = __builtin_amdgcn_alignbyte(x2, x1, sh);
        const u64 qm = ((p0 + jj) << 24) | blk4 | bb;
        /* the round's bits to lanes [xn, xn + cnt) of the batch; the other
         * lanes fill the rest, so the permute is one-to-one */
        const u32 rk = __builtin_amdgcn_mbcnt_hi((u32)(B >> 32), __builtin_amdgcn_mbcnt_lo((u32)B, 0));
        const u32 dst = have ? st.xn + rk : (st.xn + cnt + (lane - rk)) & (WAVE - 1);
        const int da = (int)(dst << 2);
        const u32 r0 = (u32)__builtin_amdgcn_ds_permute(da, (int)(u32)qm);
        const u32 r1 = (u32)__builtin_amdgcn_ds_permute(da, (int)(u32)(qm >> 32));
        const u32 r2 = (u32)__builtin_amdgcn_ds_permute(da, (int)key_lo);
        const u32 r3 = (u32)__builtin_amdgcn_ds_permute(da, (int)key_hi);
        const bool mine = lane - st.xn < cnt;
        st.xs[0] = mine ? r0 : st.xs[0];
        st.xs[1] = mine ? r1 : st.xs[1];
        st.xs[2] = mine ? r2 : st.xs[2];
        st.xs[3] = mine ? r3 : st.xs[3];
        st.xn += cnt;
    }
}

/* One 1 KiB iteration at aoff `ib`: lane l owns bytes [ib + 16 l, +16),
 * d = the lane's 16 bytes.  Every key looks back (FDR4: the two bytes before
 * a position; Teddy: the position's own byte), so no key needs the byte
 * after the chunk and an iteration never waits on the next chunk's load. */
template <int MODE, bool EDGE, bool XP, bool SPLIT>
__device__ __forceinline__ IterState lit_iter(const VsaLitParams &P, const ConfLds &cl,
                                              const LitShared &L, const SegCtx &S,
                                              u32 mis, int64_t ib, uint4 chunk,
                                              IterState in, u32 bucket_mask) {
    typedef LitTraits<MODE> T;
    typedef typename T::S_t S_t;
    const u32 lane = lane_id();
    const int64_t p0 = ib + 16 * (int64_t)lane;
    const int64_t q0 = p0 - S.blo;

    u32 d[4] = {chunk.x, chunk.y, chunk.z, chunk.w};
    /* edge iterations: readable bytes [vlo, bhi) and looked-up positions */
    u32 look_m = 0xffffu;
    if (EDGE) {
        const int r_len = rel32(S.len, q0);
        const u32 bm = range_mask(rel32(S.vlo - S.blo, q0), r_len);
#pragma unroll
        for (int w = 0; w < 4; w++) d[w] &= nib_to_bytes(bm >> (4 * w));
        look_m = range_mask(rel32(MODE == VSA_MODE_FDR4 ? S.zbase : S.qlo, q0), r_len);
    }

    constexpr bool F4 = MODE == VSA_MODE_FDR4;
    /* sweep state in lane-rotated registers (p3 / p4) */
    constexpr bool PSTATE = F4 && !EDGE;
    u32 pv3;
    IterState out;
    if constexpr (PSTATE) {
        /* lane 0: the previous chunk's lane-63 d[3], rotated in last time */
        pv3 = lane_up1_or_old(in.p3, d[3]);
        out.p3 = lane_ror1(d[3]);
    } else {
        pv3 = writelane_u32<0>(lane_up1(d[3]), (u32)(in.pbytes >> 32));
    }
    u32 c[T::CW];
    out.ncand = in.ncand;
    out.tail_cache = in.tail_cache;
    out.head = in.head;
#pragma unroll
    for (int k = 0; k < 4; k++) out.xs[k] = in.xs[k];
    out.xn = in.xn;
    if constexpr (PSTATE) {
        out.pbytes = (in.pbytes & 0xffffffff00000000ULL) | readlane_u32(d[2], WAVE - 1);
        out.carry = in.carry;
    } else {
        out.pbytes = ((u64)readlane_u32(d[3], WAVE - 1) << 32) | readlane_u32(d[2], WAVE - 1);
    }
    if constexpr (F4) {
        /* FDR4 (fdr4_conf): ends 0..15 in U[0..3] in end order; U[4] = the
         * next lane's ends 0..2 (lane 63: the next chunk's) */
        u32 U[5];
        fdr4_conf<EDGE>(L, {d[0], d[1], d[2], d[3]}, pv3, look_m, U);
        /* split passes (runtime.hip, large sets; their own kernels): this
         * pass's ends are those whose byte has bit 0 == end_par - 1; the
         * others are the other pass's, dead here */
        auto split_mask = [&]() {
            if constexpr (SPLIT) {
                const u32 fl = P.end_par == 1 ? 0u : 0x01010101u;
#pragma unroll
                for (int w = 0; w < 4; w++) {
                    const u32 t = (d[w] ^ fl) & 0x01010101u;
                    U[w] |= (t << 8) - t;
                }
            }
        };
        if constexpr (EDGE) {
            const u32 s_in = writelane_u32<0>(lane_up1(U[4]), (u32)in.carry);
            out.carry = readlane_u32(U[4], WAVE - 1);
            U[0] |= s_in;
            split_mask();
        } else {
            /* lane 0: the previous chunk's lane-63 U[4], rotated in last time */
            U[0] |= lane_up1_or_old(in.p4, U[4]);
            out.p4 = lane_ror1(U[4]);
            split_mask();
            const u32 nbm = ~bucket_mask;
            if (!wave_any(((U[0] & U[1] & U[2] & U[3]) | nbm) != 0xffffffffu)) return out;
        }
#pragma unroll
        for (int w = 0; w < 4; w++) c[w] = U[w];
    } else {
    /* Teddy / Fat Teddy: the lane's 16 lookups ... */
    S_t x[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
        /* byte r of d[w] -> address byte 1, L.tsel = 0x10000 | lane slot */
        const u32 sel = 0x0c020000u | ((4u + (j & 3)) << 8);
        const u32 a = __builtin_amdgcn_perm(d[j >> 2], L.tsel, sel);
        if constexpr (MODE == VSA_MODE_TEDDY) x[j] = lds_ld32a(a);
        else x[j] = lds_ld64(a);
        if (EDGE) {
            if (!((look_m >> j) & 1u)) x[j] = 0;
        }
    }
    /* ... OR-ed into place: field k of x[j] lands on end j + k */
    u64 s_out;
    conf_accumulate<MODE>(x, c, s_out);
    /* spill from the previous lane (lane 0: from the previous chunk) */
    const u32 s_in_lo = writelane_u32<0>(lane_up1((u32)s_out), (u32)in.carry);
    const u32 s_in_hi = sizeof(S_t) == 8
                            ? writelane_u32<0>(lane_up1((u32)(s_out >> 32)), (u32)(in.carry >> 32))
                            : 0u;
    const u64 s_in = ((u64)s_in_hi << 32) | s_in_lo;
    out.carry = ((u64)readlane_u32((u32)(s_out >> 32), WAVE - 1) << 32) |
                readlane_u32((u32)s_out, WAVE - 1);
    c[0] |= (u32)s_in;
    if constexpr (sizeof(S_t) == 8) c[1] |= (u32)(s_in >> 32);
    } /* Teddy lookups */
    if (EDGE) {
        if constexpr (MODE == VSA_MODE_FDR4) if (!S.stream) {
            /* start state: byte i applies to end start + i (the short zone
             * shifts fdr->start by 16 - (len - start) against a scan from
             * len - 16, fdr.c:372-440 and :712-720, landing on start too):
             * end q0 + j takes byte q0 + j - start of the zero-padded state */
            const int64_t r0 = q0 - S.start;
            if (r0 > -16 && r0 < 16) {
                const u32 sv[4] = {(u32)P.state_lo, (u32)(P.state_lo >> 32), (u32)P.state_hi,
                                   (u32)(P.state_hi >> 32)};
#pragma unroll
                for (int w = 0; w < 4; w++) c[w] |= window4(sv, (int)r0 + 4 * w);
            }
        }
        /* only ends in [max(start, rlo), len) are reported */
        const u32 out_m = ~range_mask(rel32(S.rlo, q0), rel32(S.len, q0)) & 0xffffu;
        if constexpr (T::LB == 8) {
#pragma unroll
            for (int w = 0; w < 4; w++) c[w] |= nib_to_bytes(out_m >> (4 * w));
        } else {
#pragma unroll
            for (int w = 0; w < 8; w++) {
                const u32 t = out_m >> (2 * w);
                c[w] |= ((t & 1u) ? 0xffffu : 0u) | ((t & 2u) ? 0xffff0000u : 0u);
            }
        }
    }

    /* candidate bits (do_confirm_fdr skips empty buckets, cf == 0): some
     * ~c[i] & bucket_mask != 0  <=>  (AND_i c[i]) | ~bucket_mask != ~0, so
     * the common no-candidate case costs an AND tree, not CW masks */
    u32 all = c[0];
#pragma unroll
    for (int i = 1; i < T::CW; i++) all &= c[i];
    if (!wave_any((all | ~bucket_mask) != 0xffffffffu)) return out;
    /* diagnostic (dbg & 32768): cycles of the candidate path before the
     * push -> counters[13], of the push (with any wait for ring room) ->
     * [14], iterations taking it -> [15] */
#ifdef VSA_DIAG
    const bool tdiag = (P.dbg & 32768) != 0;
#else
    constexpr bool tdiag = false; /* diagnostic builds only (-DVSA_DIAG) */
#endif
    const u64 t_c0 = tdiag ? __builtin_amdgcn_s_memtime() : 0;
    u32 any = 0;
#pragma unroll
    for (int i = 0; i < T::CW; i++) {
        c[i] = ~c[i] & bucket_mask;
        any |= c[i];
    }
    if (VSA_DBG(P.dbg, 32)) {
        /* diagnostic first-stage candidate count */
        u32 pc = 0;
#pragma unroll
        for (int i = 0; i < T::CW; i++) pc += __popc(c[i]);
#pragma unroll
        for (int dd = 32; dd >= 1; dd >>= 1) pc += shfl_xor_u32(pc, dd);
        out.ncand += readfirstlane_u32(pc);
    }
    if (VSA_DBG(P.dbg, 8)) return out;

    /* bytes p0-8 .. p0+15 for the 8-byte confirm keys */
    u32 pv2 = lane_up1(d[2]);
    if (lane == 0) pv2 = (u32)in.pbytes;
    /* one chunk entry per lane with candidates; the confirm wave expands it.
     * In a run the lane's block is the one holding p0 (a chunk across the
     * boundary is moved on by the confirm, confirm_multi) */
    const u32 lblk = S.blk + (p0 >= S.run_nxt ? 1u : 0u);
    const u64 meta = (u64)p0 | ((u64)lblk << ENT_BLK_SHIFT);
    if constexpr (XP) {
        xp_push(P, cl, L, out, c, meta, pv2, pv3, d);
        return out;
    }
    u32 w[4 * T::EW];
#pragma unroll
    for (int i = 0; i < 4 * T::EW; i++) w[i] = 0;
    w[0] = (u32)meta;
    w[1] = (u32)(meta >> 32);
#pragma unroll
    for (int i = 0; i < T::CW; i++) w[2 + i] = c[i];
    w[2 + T::CW] = pv2;
    w[3 + T::CW] = pv3;
#pragma unroll
    for (int i = 0; i < 4; i++) w[4 + T::CW + i] = d[i];
    const u64 t_c1 = tdiag ? __builtin_amdgcn_s_memtime() : 0;
    ring_push<T::EW>(L, out, any != 0, w);
    if (tdiag && lane == 0) {
        /* per workgroup in LDS (one global word per counter would
         * serialize every wave's add chip-wide) */
        const u64 t_c2 = __builtin_amdgcn_s_memtime();
        atomicAdd(&L.diag[0], (unsigned long long)(t_c1 - t_c0));
        atomicAdd(&L.diag[1], (unsigned long long)(t_c2 - t_c1));
        atomicAdd(&L.diag[2], 1ull);
    }
    return out;
}

/* Noodle (noodle_engine.cpp:75-134, noodle_engine_simd.hpp:173-226): end e
 * is a match when the msk_len bytes ending at e, masked, equal cmp and the
 * literal starts at or after `start`.  P.nood_msk / nood_cmp are the
 * reference msk / cmp shifted to the top of a u64, compared against the 8
 * bytes ending at e (bytes outside the block read as 0, never matched since
 * those ends are cut). */
template <bool EDGE>
__device__ __forceinline__ IterState nood_iter(const VsaLitParams &P, const LitShared &L,
                                               const SegCtx &S, int64_t ib, uint4 chunk,
                                               IterState in) {
    const u32 lane = lane_id();
    const int64_t p0 = ib + 16 * (int64_t)lane;
    const int64_t q0 = p0 - S.blo;
    u32 d[4] = {chunk.x, chunk.y, chunk.z, chunk.w};
    if (EDGE) {
        const u32 bm = range_mask(rel32(S.vlo - S.blo, q0), rel32(S.len, q0));
#pragma unroll
        for (int w = 0; w < 4; w++) d[w] &= nib_to_bytes(bm >> (4 * w));
    }
    u32 pv2 = lane_up1(d[2]), pv3 = lane_up1(d[3]);
    if (lane == 0) {
        pv2 = (u32)in.pbytes;
        pv3 = (u32)(in.pbytes >> 32);
    }
    IterState out = in;
    out.pbytes = ((u64)readlane_u32(d[3], WAVE - 1) << 32) | readlane_u32(d[2], WAVE - 1);
    if (!EDGE) {
        /* key prefilter (the reference scans for the literal's key bytes
         * before confirming, noodle_engine_simd.hpp:173-226): the last
         * three literal bytes under their masks, four positions per dword,
         * with a SWAR zero-byte test; the full compare runs only when some
         * lane has a key hit (shorter literals: the missing bytes' mask and
         * cmp are 0, always equal) */
        auto rep8 = [](u64 v, int byte) { return ((u32)(v >> (8 * byte)) & 0xffu) * 0x01010101u; };
        const u32 M2 = rep8(P.nood_msk, 7), C2 = rep8(P.nood_cmp, 7);
        const u32 M1 = rep8(P.nood_msk, 6), C1 = rep8(P.nood_cmp, 6);
        const u32 M0 = rep8(P.nood_msk, 5), C0 = rep8(P.nood_cmp, 5);
        u32 z = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const u32 lo = k ? d[k - 1] : pv3;
            const u32 p1 = __builtin_amdgcn_alignbyte(d[k], lo, 3);
            const u32 p2 = __builtin_amdgcn_alignbyte(d[k], lo, 2);
            const u32 t = or3((d[k] & M2) ^ C2, (p1 & M1) ^ C1, (p2 & M0) ^ C0);
            z |= (t - 0x01010101u) & ~t;
        }
        if (!wave_any((z & 0x80808080u) != 0)) return out;
    }
    const u32 w[6] = {pv2, pv3, d[0], d[1], d[2], d[3]};
    const u32 mlo = (u32)P.nood_msk, mhi = (u32)(P.nood_msk >> 32);
    const u32 clo = (u32)P.nood_cmp, chi = (u32)(P.nood_cmp >> 32);
    u32 hits = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int bo = j + 1; /* 8 bytes ending at p0 + j start at w byte j + 1 */
        u32 lo, hi;
        if (bo & 3) {
            lo = __builtin_amdgcn_alignbyte(w[(bo >> 2) + 1], w[bo >> 2], bo & 3);
            hi = __builtin_amdgcn_alignbyte(w[(bo >> 2) + 2], w[(bo >> 2) + 1], bo & 3);
        } else {
            lo = w[bo >> 2];
            hi = w[(bo >> 2) + 1];
        }
        if (((lo & mlo) == clo) & ((hi & mhi) == chi)) hits |= 1u << j;
    }
    if (EDGE) {
        /* noodExecStreaming (start 0): literals may begin up to
         * min(hlen, msk_len - 1) bytes into the history (noodle_engine.cpp:
         * 149-180) -- S.qlo carries that (0 in block mode) */
        const int64_t elo = S.start + (int64_t)P.nood_len - 1 + S.qlo;
        hits &= range_mask(rel32(elo > S.rlo ? elo : S.rlo, q0), rel32(S.len, q0));
    }
    if (!wave_any(hits != 0)) return out;
    const u64 meta = (u64)p0 | ((u64)S.blk << ENT_BLK_SHIFT);
    const u32 ent[8] = {(u32)meta, (u32)(meta >> 32), 0, 0, hits, 0, 0, 0};
    ring_push<2>(L, out, hits != 0, ent);
    return out;
}

template <int MODE, bool EDGE, bool XP, bool SPLIT>
__device__ __forceinline__ IterState scan_iter(const VsaLitParams &P, const ConfLds &cl,
                                               const LitShared &L, const SegCtx &S,
                                               u32 mis, int64_t ib, uint4 chunk,
                                               IterState in, u32 bucket_mask) {
    if constexpr (MODE == VSA_MODE_NOOD) {
        return nood_iter<EDGE>(P, L, S, ib, chunk, in);
    } else {
        return lit_iter<MODE, EDGE, XP, SPLIT>(P, cl, L, S, mis, ib, chunk, in,
                                                   bucket_mask);
    }
}

__device__ __forceinline__ uint4 load_chunk(const u8 *A, int64_t p0, int64_t bhi) {
    uint4 v = make_uint4(0, 0, 0, 0);
    typedef u32 v4u __attribute__((ext_vector_type(4)));
    if (p0 < bhi) {
        v4u t = __builtin_nontemporal_load((const v4u *)(A + p0));
        v = make_uint4(t.x, t.y, t.z, t.w);
    }
    return v;
}

/* unconditional 16-byte load (caller guarantees the address is valid) */
__device__ __forceinline__ uint4 load_chunk_nc(const u8 *A, int64_t p0) {
    typedef u32 v4u __attribute__((ext_vector_type(4)));
    v4u t = __builtin_nontemporal_load((const v4u *)(A + p0));
    return make_uint4(t.x, t.y, t.z, t.w);
}

/* unconditional wave load of the 1 KiB at A + ib (wave-uniform ib): lane l
 * reads bytes [16 l, 16 l + 16).  The base goes through SGPRs so the load
 * is an saddr global_load_dwordx4 with a 32-bit lane offset (no per-lane
 * 64-bit address arithmetic in the sweep). */
__device__ __forceinline__ const u8 *uniform_ptr(const u8 *p) {
    const u64 a = (u64)p;
    return (const u8 *)(((u64)readfirstlane_u32((u32)(a >> 32)) << 32) |
                        readfirstlane_u32((u32)a));
}
__device__ __forceinline__ uint4 load_wave_kib(const u8 *base, u32 off) {
    typedef u32 v4u __attribute__((ext_vector_type(4)));
    /* global address space: a flat load would also count in lgkmcnt and
     * serialize against the table's LDS reads */
    typedef const __attribute__((address_space(1))) v4u gv4u;
    gv4u *p = (gv4u *)(base + (off + 16 * lane_id()));
    v4u t = __builtin_nontemporal_load(p);
    return make_uint4(t.x, t.y, t.z, t.w);
}

#define LIT_DEPTH 4 /* chunks in flight per scanning wave (1 KiB each) */
/* s_waitcnt immediate (gfx9 encoding): vmcnt 0, expcnt and lgkmcnt left at
 * their maximum (no wait) */
#define VMCNT0 0x0f70

/* A workgroup's confirm wave (one, or several for large literal sets, each
 * serving every nc-th ring): gathers up to 64 chunk entries per round from
 * its rings (each consumed in order), expands their candidate bits one per
 * lane per round, drops the candidates whose litIndex slot is empty (LDS
 * slot bitmap: litIndex[hash] == 0 means no LitInfo chain,
 * fdr_confirm_runtime.h:55-58), queues the rest in its private LDS queue and
 * runs the exact confirm CONF_U x 64 at a time.  Its global-memory latency
 * never stalls a scanning wave.  Exits once every scanning wave has finished
 * (q_done, read before the heads), every ring is empty and the queue is
 * drained.  (A two-step expansion -- all bits written as keys to a
 * pre-filter queue by their lanes, then filtered 64 at a time with every
 * lane busy -- measured slower: 10.4 vs 9.4 ms at 20k literals.) */
#define MAX_CONF_WAVES 4
#ifndef CONF_IDLE_SLEEP
#define CONF_IDLE_SLEEP 8 /* s_sleep units (64 clocks) between idle polls */
#endif
#define EXP_U 1 /* candidate bits per lane per expansion round (2 and 4 measured
                   slower at 5k and at 20k literals) */
/* confirm queue entries of a confirm wave confirming CU per lane per batch:
 * >= CU * 64 + EXP_U * 64 - 1 (a round adds <= EXP_U * 64), a power of two */
#define PQ_ENTRIES(CU) ((CU) == 4 ? 512 : 256)
template <int MODE, int CONF_U, bool XP>
__device__ __forceinline__ void confirm_wave(const VsaLitParams &P, const ConfLds &cl,
                                             const uint4 *rings, u32 lg, u32 *tails,
                                             const u32 *heads, const u32 *q_done, u32 mis,
                                             const u32 *slots, QEnt *pq, u32 cw, u32 nc,
                                             u64 *pcl, u64 (&dg)[3]) {
    typedef LitTraits<MODE> T;
    constexpr int EW = XP ? 1 : T::EW; /* ring entry: chunk or QEnt (XP) */
    constexpr int CW = T::CW;
    constexpr u32 PQ_CAP = PQ_ENTRIES(CONF_U);
    static_assert(PQ_CAP >= CONF_U * 64 + EXP_U * 64 - 1, "confirm queue too small");
    const u32 lane = lane_id();
    const u32 cap = 1u << lg;
    /* confirm wave cw of nc serves rings cw, cw + nc, ... (nr of them): lane
     * sl * i + k reads slot tail + k of ring rr = cw + nc i, sl = the slots
     * per ring one gather reads (64 / nr lanes, at most the ring size) */
    const u32 nscan = LIT_WAVES - nc;
    const u32 nr = (nscan - cw + nc - 1) / nc;
    const u32 sl0 = nr <= 4 ? 16u : nr <= 8 ? 8u : 4u;
    const u32 sl = sl0 < cap ? sl0 : cap;
    const u32 ri = lane / sl;
    const u32 rr = cw + nc * ri, rk = lane - ri * sl;
    const bool ring_lane = ri < nr;
    u32 tail = 0; /* ring rr's consumed position (same in its 4 lanes) */
    u32 filled = 0;
    u32 consumed = 0;
    u32 pq_head = 0, pq_tail = 0; /* confirm queue cursors (wave-uniform) */
    /* VSA_DEBUG_FLAGS bit 6: cycles per phase + counts -> counters[4..11],
     * kept in LDS (pcl, this wave's 8 slots) so they hold no registers */
    const bool prof = VSA_DBG(P.dbg, 64);
    u64 tmark = prof ? __builtin_amdgcn_s_memtime() : 0;
    auto pcount = [&](int i, u64 v) {
        if (prof && lane == 0) pcl[i] += v;
    };
    auto phase = [&](int i) {
        if (prof) {
            const u64 now = __builtin_amdgcn_s_memtime();
            pcount(i, now - tmark);
            tmark = now;
        }
    };
    /* confirm k <= CONF_U * 64 queued candidates, CONF_U per lane */
    /* diagnostic (dbg & 8192, wave log): when every scanning wave was first
     * seen done, when the last batch started, batches after that */
#ifdef VSA_DIAG
    const bool dlog = (P.dbg & 8192) != 0;
#else
    constexpr bool dlog = false; /* diagnostic builds only (-DVSA_DIAG) */
#endif
    bool seen_done = false;
    auto confirm_batch = [&](u32 k) {
        if (dlog) {
            dg[1] = __builtin_amdgcn_s_memrealtime();
            if (seen_done) dg[2]++;
        }
        phase(1);
        asm volatile("" ::: "memory");
        QEnt q[CONF_U];
        bool valid[CONF_U];
#pragma unroll
        for (int i = 0; i < CONF_U; i++) {
            const u32 j = lane + (u32)WAVE * i;
            valid[i] = j < k;
            q[i] = valid[i] ? pq[(pq_tail + j) & (PQ_CAP - 1)] : QEnt{0, 0};
        }
        confirm_multi<CONF_U>(P, cl, q, valid, mis); /* every lane: wave-uniform inside */
        asm volatile("" ::: "memory");
        pq_tail += k;
        consumed += k;
        pcount(7, 1);
        phase(2);
    };
    for (;;) {
        const bool all_done = lds_ld32(q_done) == nscan;
        asm volatile("" ::: "memory");
        if (dlog && all_done && !seen_done) {
            seen_done = true;
            dg[0] = __builtin_amdgcn_s_memrealtime();
        }
        /* poll: the served rings' heads in one read */
        const u32 avail = ring_lane ? lds_ld32(&heads[rr]) - tail : 0u;
        const bool valid = rk < avail;
        u32 e[4 * EW];
#pragma unroll
        for (int i = 0; i < 4 * EW; i++) e[i] = 0;
        filled = (u32)__popcll(__ballot(valid));
        if (filled) {
            /* gather the available slots (up to sl per ring) */
            if (valid) {
                const uint4 *q = rings + ((size_t)rr * cap + ((tail + rk) & (cap - 1))) * EW;
#pragma unroll
                for (int k = 0; k < EW; k++) {
                    const uint4 v = q[k];
                    e[4 * k] = v.x;
                    e[4 * k + 1] = v.y;
                    e[4 * k + 2] = v.z;
                    e[4 * k + 3] = v.w;
                }
            }
            asm volatile("" ::: "memory"); /* entries read before they are freed */
            const u32 run = avail < sl ? avail : sl;
            tail += run;
            if (rk == 0 && ring_lane && run) lds_st32(&tails[rr], tail);
        }
        pcount(4, 1);
        pcount(5, filled);
        phase(0);
        if (filled == 0) {
            if (pq_head != pq_tail) {
                confirm_batch(pq_head - pq_tail); /* < CONF_U * 64 queued */
                continue;
            }
            if (all_done) break;
            /* idle: yield issue priority while polling */
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_s_sleep(CONF_IDLE_SLEEP);
            phase(3);
            continue;
        }
        if (VSA_DBG(P.dbg, 128)) continue; /* experiment: drop gathered entries */
        if constexpr (XP) {
            /* QEnt entries (scanner expansion): queue them and confirm */
            const u64 pm = __ballot(valid);
            if (valid) {
                const u32 r = __builtin_amdgcn_mbcnt_hi((u32)(pm >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((u32)pm, 0));
                QEnt *q = &pq[(pq_head + r) & (PQ_CAP - 1)];
                q->meta = ((u64)e[1] << 32) | e[0];
                q->key = ((u64)e[3] << 32) | e[2];
            }
            pq_head += filled;
            /* < CONF_U * 64 queued before, <= 64 added */
            if (pq_head - pq_tail >= (u32)WAVE * CONF_U) {
                if (filled >= 16 && !VSA_DBG(P.dbg, 1024)) __builtin_amdgcn_s_setprio(2);
                else __builtin_amdgcn_s_setprio(0);
                confirm_batch(WAVE * CONF_U);
            }
            continue;
        }
        /* a backlog (many entries per gather): issue ahead of the scanners
         * on this SIMD (the youngest wave otherwise loses VALU arbitration
         * to all of them), as large literal sets need; a light load runs at
         * base priority, which measured 1.5 % faster at cfg 4.  Noodle
         * entries are final matches, where priority measured slower. */
        if constexpr (MODE != VSA_MODE_NOOD)
        {
            if (filled >= 16 && !VSA_DBG(P.dbg, 1024)) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(0);
        }
        const u64 meta0 = ((u64)e[1] << 32) | e[0];
        const u64 p0 = meta0 & ENT_P0_MASK;
        const u32 blk = (u32)(meta0 >> ENT_BLK_SHIFT);
        if constexpr (MODE == VSA_MODE_NOOD) {
            /* noodle hits are final: emit (end, id) */
            u32 hits = e[4];
            /* one atomic per lane with hits (measured faster here than a
             * wave prefix sum + one atomic per gather) */
            if (hits && P.bin_keys) {
                /* staged binned sort: the hits straight into their bins,
                 * counted in LDS (no output slot, no shared global word) */
                __hip_atomic_fetch_add(const_cast<u32 *>(&cl.nrec), (u32)__popc(hits),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                consumed += (u32)__popc(hits);
                for (; hits; hits &= hits - 1) {
                    const u32 j = __ffs(hits) - 1;
                    const u64 end = p0 + j - mis;
                    const u32 bin = rec_bin(P, cl, end);
                    const u32 s = bin_slot_take(P, cl, bin);
                    if (s < VSA_SORT_BIN_MAX) {
                        const size_t q = bin_row(P, bin) * VSA_SORT_BIN_MAX + s;
                        P.bin_keys[q] = end << VSA_KEY_END_SHIFT;
                        P.bin_ids[q] = P.nood_id;
                    } else {
                        flag_crowd(P);
                    }
                }
            } else if (hits) {
                /* one atomic per lane with hits (measured faster here than
                 * a wave prefix sum + one atomic per gather) */
                const u32 n = (u32)__popc(hits);
                unsigned long long slot = atomicAdd(&P.counters[0], (unsigned long long)n);
                consumed += n;
                for (; hits; hits &= hits - 1, slot++) {
                    const u32 j = __ffs(hits) - 1;
                    if (slot < P.out_cap) {
                        P.out_keys[slot] = (p0 + j - mis) << VSA_KEY_END_SHIFT;
                        P.out_ids[slot] = P.nood_id;
                    }
                }
            }
            continue;
        } else {
            u32 c[CW];
#pragma unroll
            for (int i = 0; i < CW; i++) c[i] = e[2 + i];
            const u64 W0 = ((u64)e[3 + CW] << 32) | e[2 + CW];
            const u64 W1 = ((u64)e[5 + CW] << 32) | e[4 + CW];
            const u64 W2 = ((u64)e[7 + CW] << 32) | e[6 + CW];
            /* Wave-uniform loop: each round every lane takes its EXP_U
             * lowest remaining candidate bits (over all conf words), so the
             * prefilter's dependent LDS reads (bucket record, slot word) of
             * up to 4 x 64 candidates are in flight together. */
            for (;;) {
                bool have[EXP_U];
                u32 jj[EXP_U], bb[EXP_U];
#pragma unroll
                for (int u = 0; u < EXP_U; u++) {
                    u32 word = 0, bits = c[0];
#pragma unroll
                    for (int k = 1; k < CW; k++) {
                        const bool take = bits == 0;
                        bits = take ? c[k] : bits;
                        word = take ? (u32)k : word;
                    }
                    have[u] = bits != 0;
                    const u32 bit = __ffs(bits) - 1;
#pragma unroll
                    for (int k = 0; k < CW; k++)
                        if (have[u] && word == (u32)k) c[k] &= c[k] - 1;
                    if constexpr (T::LB == 8) {
                        jj[u] = 4 * word + (bit >> 3);
                        bb[u] = bit & 7;
                    } else {
                        jj[u] = 2 * word + (bit >> 4);
                        bb[u] = bit & 15;
                    }
                }
                if (!__any(have[0])) break;
                pcount(6, 1);
                u64 key[EXP_U];
                PfRec pf[EXP_U];
#pragma unroll
                for (int u = 0; u < EXP_U; u++) {
                    /* key = bytes [j-7, j] = byte offset j+1 .. j+8 of W0:W1:W2 */
                    const u32 o = jj[u] + 1;
                    u64 k8;
                    if (o < 8) k8 = (W0 >> (8 * o)) | (W1 << (64 - 8 * o));
                    else if (o == 8) k8 = W1;
                    else if (o < 16) k8 = (W1 >> (8 * (o - 8))) | (W2 << (64 - 8 * (o - 8)));
                    else k8 = W2;
                    key[u] = k8;
                    /* unconditional reads (bb in range either way), so the
                     * EXP_U reads of each kind are in flight together */
                    pf[u] = cl.pf[bb[u] & 15];
                }
                u32 sw[EXP_U], sh[EXP_U];
                bool chk[EXP_U];
#pragma unroll
                for (int u = 0; u < EXP_U; u++) {
                    /* LDS slot-bitmap prefilter: litIndex[hash] == 0 rejects */
                    chk[u] = have[u] && pf[u].slot_off != 0xffffffffu;
                    const u32 h = (u32)(((key[u] & pf[u].andmsk) * P.pf_mult) >> pf[u].shift);
                    sh[u] = h & 31;
                    sw[u] = chk[u] ? lds_ld32(&slots[pf[u].slot_off + (h >> 5)]) : ~0u;
                }
                bool push[EXP_U];
#pragma unroll
                for (int u = 0; u < EXP_U; u++) {
                    push[u] = have[u] && ((sw[u] >> sh[u]) & 1u);
                    if (VSA_DBG(P.dbg, 16)) push[u] = false;
                }
#pragma unroll
                for (int u = 0; u < EXP_U; u++) {
                    const u64 pm = __ballot(push[u]);
                    if (push[u]) {
                        const u32 r = __builtin_amdgcn_mbcnt_hi(
                            (u32)(pm >> 32), __builtin_amdgcn_mbcnt_lo((u32)pm, 0));
                        QEnt *q = &pq[(pq_head + r) & (PQ_CAP - 1)];
                        q->meta = ((p0 + jj[u]) << 24) | ((u64)blk << 4) | bb[u];
                        q->key = key[u];
                    }
                    pq_head += (u32)__popcll(pm);
                }
                /* < 256 queued before the round, <= 4 x 64 added: one batch
                 * brings the queue back under 256 (PQ_CAP 512) */
                if (pq_head - pq_tail >= (u32)WAVE * CONF_U) confirm_batch(WAVE * CONF_U);
            }
            phase(1);
        }
    }
    /* confirm-stage candidates (first-stage count instead under dbg & 32) */
    if (P.counters && lane == 0 && consumed && !VSA_DBG(P.dbg, 32)) {
        atomicAdd(&P.counters[2], (unsigned long long)consumed);
        if (P.fin_keys)
            __hip_atomic_fetch_add(const_cast<u32 *>(&cl.f_cand), consumed, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (prof && lane == 0) {
        phase(1);
        for (int i = 0; i < 8; i++) atomicAdd(&P.counters[4 + i], (unsigned long long)pcl[i]);
    }
}

/* dst[i] = src(i) for i < n, thread tid of LIT_THREADS: UNR loads issued
 * before their LDS stores (a plain strided loop waits out one memory round
 * trip per step: ~8 of them for a 128 KiB table at every launch) */
template <int UNR, typename TV, typename F>
__device__ __forceinline__ void stage_lds(TV *dst, u32 n, u32 tid, F &&src) {
    /* full rounds: UNR loads issued back to back, then the stores.  (With a
     * bound check on every load the compiler waited for each load before
     * issuing the next -- the 128 KiB FDR4 table took 8 serial memory round
     * trips, ~3 us of every launch's start.) */
    u32 base = 0;
    for (; base + UNR * LIT_THREADS <= n; base += UNR * LIT_THREADS) {
        TV v[UNR];
#pragma unroll
        for (int k = 0; k < UNR; k++) v[k] = src(base + (u32)k * LIT_THREADS + tid);
#pragma unroll
        for (int k = 0; k < UNR; k++) dst[base + (u32)k * LIT_THREADS + tid] = v[k];
    }
    for (u32 i = base + tid; i < n; i += LIT_THREADS) dst[i] = src(i);
}

__device__ __forceinline__ void fused_finish(const VsaLitParams &P, const ConfLds &cl, u32 *sc);

/* ---- dynamic shares (VsaLitParams.dyn_kib) ----
 * The XCDs of a box drift apart and back over a few launches (XCD pairs
 * 20-40 us apart on a 4 GiB scan, the deviation's correlation 0.92 from one
 * launch to the next and 0.6 four launches later:
 * profiles/r06/r06y_fb_trace_*.txt), faster than host-side feedback, which
 * rebuilds the plan, can follow.  So each launch sets its own shares: wave
 * 0 of every workgroup reads the previous launch's end times and weights
 * (one memory round trip, beside the table staging), derives per-XCD
 * weights that would have ended its XCDs together, and cuts the plan's
 * live KiB at the weighted prefix sums.  Every workgroup computes the same
 * boundaries from the same inputs with the same instructions (integer
 * prefix sums and division; the float part runs on wave-uniform values in
 * one order), so workgroup b's upper boundary is b + 1's lower one and
 * every KiB is scanned exactly once.  Each boundary stays within dyn_margin
 * KiB of the equal-share one, which the host's owned sort bins exclude
 * (plan.hip plan_wg_bins).  The segments are the host list's (parts of
 * large blocks only); a workgroup takes those overlapping its range,
 * clipped to it. */
struct DynB {
    u32 s_lo, s_hi; /* the workgroup's segments [s_lo, s_hi) */
    u32 lk, hk;     /* its KiB range */
};

__device__ __forceinline__ u32 wave_sum_u32(u32 v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += shfl_xor_u32(v, m);
    return readfirstlane_u32(v);
}

/* The segments whose KiB position (descriptor word 3, ascending) is <= L
 * (or < L), counted over a 64-entry window loaded at the kernel's entry
 * around the equal-share boundary's segment (the boundary moves at most
 * 1/6 of a share, a few segments), else by a 64-way search of the list. */
__device__ __forceinline__ u32 dyn_window_base(u32 n, u32 near) {
    u32 base = near > 32 ? near - 32 : 0;
    if (base + 64 > n) base = n > 64 ? n - 64 : 0;
    return base;
}

__device__ __forceinline__ u32 dyn_count(const VsaLitParams &P, u32 lane, u32 base, u32 v, u32 L,
                                         bool strict) {
    const u32 n = (u32)P.nsegs;
    const u32 *pos = P.seg_desc + 3;
    auto pred = [&](u32 s, u32 end) -> bool {
        if (s >= end) return false;
        const u32 x = pos[4 * (size_t)s];
        return strict ? x < L : x <= L;
    };
    {
        const bool in = base + lane < n && (strict ? v < L : v <= L);
        const u32 c = (u32)__popcll(__ballot(in));
        if ((c > 0 || base == 0) && (c < 64 || base + 64 >= n)) return base + c;
    }
    /* the count A lies in [lo, hi]: elements below lo hold, from hi on not */
    u32 lo = 0, hi = n;
    while (hi - lo > 64) {
        const u32 step = (hi - lo + 63) / 64;
        const u32 c = (u32)__popcll(__ballot(pred(lo + lane * step, hi)));
        if (c == 0) return lo;
        const u32 nhi = min(hi, lo + c * step);
        lo = lo + (c - 1) * step + 1;
        hi = nhi;
    }
    return lo + (u32)__popcll(__ballot(pred(lo + lane, hi)));
}

/* loaded by wave 0 at the kernel's entry, so the round trip overlaps the
 * table staging: the previous launch's records and weights, and the
 * segment positions around this workgroup's equal-share boundaries */
struct DynPre {
    unsigned long long en[4], ex[4];
    u32 wp;
    u32 base_lo, base_hi, v_lo, v_hi;
};

__device__ __forceinline__ void dyn_load(const VsaLitParams &P, u32 lane, DynPre &d) {
    const u32 G = gridDim.x, b = blockIdx.x;
    const u32 n = (u32)P.nsegs;
    const unsigned long long T = P.dyn_kib;
    const u32 *pos = P.seg_desc + 3;
    d.base_lo = dyn_window_base(n, (u32)((unsigned long long)n * (T * b / G) / T));
    d.base_hi = dyn_window_base(n, (u32)((unsigned long long)n * (T * (b + 1) / G) / T));
    d.v_lo = d.base_lo + lane < n ? pos[4 * (size_t)(d.base_lo + lane)] : 0xffffffffu;
    d.v_hi = d.base_hi + lane < n ? pos[4 * (size_t)(d.base_hi + lane)] : 0xffffffffu;
    constexpr unsigned long long M60 = (1ull << 60) - 1;
    d.wp = 65536;
    if (!P.dyn_prev) return;
    if (lane < 8 && P.dyn_wprev) d.wp = P.dyn_wprev[lane];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const u32 k = lane + 64 * j;
        d.en[j] = ~0ull; /* past the grid: no part in the minimum */
        d.ex[j] = M60;
        if (k < G) {
            d.ex[j] = P.dyn_prev[k];
            d.en[j] = P.dyn_prev[G + k];
        }
    }
}

/* wave 0 of each workgroup: its range and segments (grid <= 256) */
__device__ __forceinline__ void dyn_bounds(const VsaLitParams &P, u32 lane, const DynPre &dp,
                                           DynB &o) {
    const u32 G = gridDim.x, b = blockIdx.x;
    constexpr u32 ONE = 65536;
    constexpr unsigned long long M60 = (1ull << 60) - 1;
    u32 wq[8];
#pragma unroll
    for (int x = 0; x < 8; x++) wq[x] = ONE;
    u32 xk[4] = {0, 0, 0, 0};
    if (P.dyn_prev) {
        const unsigned long long *en = dp.en, *ex = dp.ex;
        const u32 wp = dp.wp;
        unsigned long long t0 = ~0ull;
        bool bad = false; /* a workgroup without a complete record */
#pragma unroll
        for (int j = 0; j < 4; j++) {
            bad = bad || !en[j] || !(ex[j] & M60);
            t0 = en[j] < t0 ? en[j] : t0;
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            const unsigned long long o2 = ((unsigned long long)shfl_xor_u32((u32)(t0 >> 32), m) << 32) |
                                          shfl_xor_u32((u32)t0, m);
            t0 = o2 < t0 ? o2 : t0;
        }
        u32 s[8], c[8];
#pragma unroll
        for (int x = 0; x < 8; x++) s[x] = c[x] = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const u32 k = lane + 64 * j;
            const u32 x = (u32)(ex[j] >> 60) & 7u;
            const unsigned long long e = ex[j] & M60;
            bad = bad || (k < G && e <= t0);
            const unsigned long long dt = e > t0 ? e - t0 : 0ull;
            const u32 d = dt < 0xffffffull ? (u32)dt : 0xffffffu;
            xk[j] = x;
#pragma unroll
            for (int xx = 0; xx < 8; xx++)
                if (k < G && x == (u32)xx) {
                    s[xx] += d;
                    c[xx] += 1;
                }
        }
        if (!__ballot(bad)) {
            float tx[8], tm = 0.f, np = 0.f;
#pragma unroll
            for (int x = 0; x < 8; x++) {
                s[x] = wave_sum_u32(s[x]);
                c[x] = wave_sum_u32(c[x]);
                tx[x] = c[x] ? (float)s[x] / (float)c[x] : 0.f;
                if (c[x]) {
                    tm += tx[x];
                    np += 1.f;
                }
            }
            tm /= np;
            /* the weights that would have ended every XCD together (time
             * per XCD ~ weight / rate), normalized to mean 1, held in
             * 0.9-1.1 */
            float tw[8], tsum = 0.f;
#pragma unroll
            for (int x = 0; x < 8; x++) {
                const float w0 = (float)readlane_u32(wp, x) * (1.f / 65536.f);
                tw[x] = c[x] ? w0 * tm / fmaxf(tx[x], 1.f) : 0.f;
                tsum += tw[x];
            }
            const float mean = tsum / np;
#pragma unroll
            for (int x = 0; x < 8; x++)
                if (c[x]) wq[x] = (u32)(fminf(1.1f, fmaxf(0.9f, tw[x] / mean)) * 65536.f + 0.5f);
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) xk[j] = 0;
        }
    }
    if (b == 0 && lane < 8 && P.dyn_wout) {
        u32 w = wq[0];
#pragma unroll
        for (int x = 1; x < 8; x++) w = lane == (u32)x ? wq[x] : w;
        P.dyn_wout[lane] = w;
    }
    /* integer prefix sums of the workgroups' weights */
    u32 pre = 0, mine = 0, tot = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const u32 k = lane + 64 * j;
        u32 w = wq[0];
#pragma unroll
        for (int x = 1; x < 8; x++) w = xk[j] == (u32)x ? wq[x] : w;
        if (k < G) {
            tot += w;
            if (k < b) pre += w;
            if (k == b) mine = w;
        }
    }
    pre = wave_sum_u32(pre);
    mine = wave_sum_u32(mine);
    tot = wave_sum_u32(tot);
    const unsigned long long T = P.dyn_kib, M = P.dyn_margin;
    auto bound = [&](u32 i, u32 S) -> u32 {
        if (i == 0) return 0u;
        if (i >= G) return (u32)T;
        const unsigned long long nom = T * i / G;
        unsigned long long L = T * S / tot;
        const unsigned long long lo = nom > M ? nom - M : 0ull, hi = min(nom + M, T);
        L = L < lo ? lo : L > hi ? hi : L;
        return (u32)L;
    };
    o.lk = bound(b, pre);
    o.hk = bound(b + 1, pre + mine);
    o.s_lo = o.s_hi = 0;
    if (o.lk < o.hk) {
        o.s_lo = dyn_count(P, lane, dp.base_lo, dp.v_lo, o.lk, false) - 1;
        o.s_hi = dyn_count(P, lane, dp.base_hi, dp.v_hi, o.hk, true);
    }
}

template <int MODE, bool XP, bool SPLIT>
__global__ void __launch_bounds__(LIT_THREADS)
vsa_lit_scan(VsaLitParams P) {
    typedef LitTraits<MODE> T;
    /* uint4 words per ring entry: a chunk entry, or a QEnt (XP) */
    constexpr int REW = XP ? 1 : T::EW;
    typedef typename T::S_t S_t;
    extern __shared__ __align__(16) u8 smem[];
    __shared__ ConfLds cl;
    __shared__ u32 q_tails[16], q_heads[16], q_done, wg_ctr, conf_fin;
    __shared__ u32 dyn_s[4]; /* dynamic shares: DynB of this workgroup */
    /* work stealing (dynamic 2): per scanning wave, the sweep groups of its
     * current segment it has not claimed yet: seg << 40 | end << 20 | cur
     * (groups of LIT_DEPTH iterations; cur = the next group to claim) */
    __shared__ unsigned long long rng[16];
    __shared__ u64 prof_lds[8 * MAX_CONF_WAVES]; /* confirm-wave profile (dbg & 64) */
    __shared__ unsigned long long diag_lds[3];   /* candidate-path cycles (dbg & 32768) */
    const u32 tid = threadIdx.x;
    const u32 lane = lane_id();
    /* provably wave-uniform: the confirm wave's s_setprio is a scalar
     * instruction that an EXEC-masked branch would run in every wave */
    const u32 wave = readfirstlane_u32(tid / WAVE);
    /* diagnostic (dbg & 8192, wave log): the kernel's entry, before staging */
    const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();
    DynPre dpre;
    if (P.dyn_kib && wave == 0) dyn_load(P, lane, dpre);

    const u32 mis = (u32)((uintptr_t)P.data & 15);
    const u8 *A = P.data - mis;

    /* ---- stage tables into LDS ---- */
    u32 tab_bytes = 0;
    const void *tab;
    if constexpr (MODE == VSA_MODE_FDR4) {
        tab_bytes = P.table_entries * 4;
        const uint4 *src = (const uint4 *)P.table;
        stage_lds<8>((uint4 *)smem, tab_bytes / 16, tid, [&](u32 i) { return src[i]; });
        tab = smem;
    } else if constexpr (MODE == VSA_MODE_NOOD) {
        tab = nullptr;
    } else {
        /* Teddy / Fat Teddy: the byte table (u64 entries) at LDS 0x10000,
         * one copy per lane & 31, so a lane group's lookups hit distinct
         * bank pairs and the address of byte c is 0x10000 | c << 8 |
         * (lane & 31) << 3: one v_perm (TEDDY_TAB_LDS) */
        u8 *tb = smem + (TEDDY_TAB_LDS - (u32)(uintptr_t)(lds_u8_t *)smem);
        if constexpr (MODE == VSA_MODE_TEDDY) {
            /* u32 entries (the low 4 fields), 32 copies in the first 128 B
             * of a 256-B row per byte value: one v_perm builds the address */
            u32 *t32 = (u32 *)tb;
            for (u32 b0 = 0; b0 < 256 * 32; b0 += 8 * LIT_THREADS) {
                u32 v[8];
#pragma unroll
                for (int k = 0; k < 8; k++) v[k] = (u32)P.table[(b0 + k * LIT_THREADS + tid) >> 5];
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const u32 i = b0 + k * LIT_THREADS + tid;
                    t32[((i >> 5) << 6) | (i & 31)] = v[k];
                }
            }
        } else {
            stage_lds<8>((u64 *)tb, 256 * 32, tid, [&](u32 i) { return P.table[i >> 5]; });
        }
        tab = tb;
    }
    /* one ring of qcap entries per scanning wave, the slot bitmaps, then the
     * confirm waves' private queues (one of 512 entries, or nconf of 256) */
    const u32 NC = P.nconf;
    const u32 NS = LIT_WAVES - NC;
    uint4 *rings = (uint4 *)(smem + ((tab_bytes + 15) & ~15u));
    u32 *slots = (u32 *)(rings + (size_t)NS * P.qcap * REW);
    QEnt *pqx = (QEnt *)(slots + ((P.slot_words + 3) & ~3u));
    stage_lds<4>(slots, P.slot_words, tid, [&](u32 i) { return P.slotmap[i]; });
    if (tid < 16) {
        const u32 off = P.conf_off[tid];
        cl.off[tid] = off;
        PfRec pf;
        pf.slot_off = P.slot_off[tid];
        if (off) {
            const u8 *fc = P.conf_base + off;
            cl.andmsk[tid] = pf.andmsk = *(const u64 *)fc;
            cl.mult[tid] = *(const u64 *)(fc + 8);
            cl.nbits[tid] = *(const u32 *)(fc + 16);
            pf.shift = 64 - (P.slot_bits[tid] ? P.slot_bits[tid] : cl.nbits[tid]);
            /* the prefilter hashes with the kernel-wide multiplier */
            if (cl.mult[tid] != P.pf_mult) pf.slot_off = 0xffffffffu;
        } else {
            cl.andmsk[tid] = pf.andmsk = 0;
            cl.mult[tid] = 0;
            cl.nbits[tid] = 1;
            pf.shift = 63;
            pf.slot_off = 0xffffffffu;
        }
        cl.pf[tid] = pf;
    }
    {
        /* owned sort bins: their counts so far (0, or the first split
         * pass's) into LDS */
        u32 lo = 0, n = 0;
        if (P.fin_keys) {
            /* fused finish: local bins over this workgroup's ends, from 0 */
            const uint32_t *f = P.fin_wg + 4 * (size_t)blockIdx.x;
            n = f[3];
            if (tid == 0) {
                cl.f_lo = ((u64)f[1] << 32) | f[0];
                cl.f_shift = f[2];
                cl.f_bad = 0;
                cl.f_cand = 0;
            }
            for (u32 i = tid; i < n; i += LIT_THREADS) cl.lbins[i] = 0;
        } else if (P.bin_keys && P.wg_bins) {
            lo = P.wg_bins[2 * blockIdx.x];
            n = P.wg_bins[2 * blockIdx.x + 1] - lo;
            for (u32 i = tid; i < n; i += LIT_THREADS) cl.lbins[i] = P.bin_counts[lo + i];
        }
        if (tid == 0) {
            cl.lb_lo = lo;
            cl.lb_n = n;
            cl.nrec = 0;
            conf_fin = 0;
        }
    }
    if (tid < 16) {
        q_tails[tid] = 0;
        q_heads[tid] = 0;
        rng[tid] = 0;
    }
    if (tid == 0) {
        q_done = 0;
        wg_ctr = 0;
        /* the schedule's feedback (runtime.hip xcd_feedback): this
         * workgroup's entry time */
        if (P.wg_time) /* atomic: the fused finish's publisher reads it */
            __hip_atomic_store(&P.wg_time[gridDim.x + blockIdx.x], t_entry, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid < 8 * MAX_CONF_WAVES) prof_lds[tid] = 0;
    if (tid < 3) diag_lds[tid] = 0;
    if (P.dyn_kib && wave == 0) {
        /* dynamic shares: this workgroup's range and segments */
        DynB d;
        dyn_bounds(P, lane, dpre, d);
        if (lane == 0) {
            dyn_s[0] = d.s_lo;
            dyn_s[1] = d.s_hi;
            dyn_s[2] = d.lk;
            dyn_s[3] = d.hk;
        }
    }
    __syncthreads();

    if (wave >= NS) {
        const u32 cw = wave - NS;
        u64 dg[3] = {0, 0, 0};
        if (NC == 1)
            confirm_wave<MODE, 4, XP>(P, cl, rings, 31 - __clz(P.qcap), q_tails, q_heads, &q_done,
                                  mis, slots, pqx, 0, 1, prof_lds, dg);
        else
            confirm_wave<MODE, 2, XP>(P, cl, rings, 31 - __clz(P.qcap), q_tails, q_heads, &q_done,
                                  mis, slots, pqx + (size_t)cw * PQ_ENTRIES(2), cw, NC,
                                  prof_lds + 8 * cw, dg);
        {
            /* the last confirm wave out stores the owned bins' counts: the
             * acq_rel add orders every confirm wave's LDS adds (lbins, nrec;
             * nrec's add returns nothing and nothing else waits on it) before
             * its own, and the last wave's reads after all of them */
            u32 prev = 0;
            if (lane == 0)
                prev = __hip_atomic_fetch_add(&conf_fin, 1u, __ATOMIC_ACQ_REL,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
            if (readfirstlane_u32(prev) + 1 == NC) {
                const u32 lo = cl.lb_lo, n = P.fin_keys ? 0u : cl.lb_n; /* fused: kept in LDS */
                for (u32 i = lane; i < n; i += WAVE) P.bin_counts[lo + i] = cl.lbins[i];
                /* the workgroup's record count: one add, not one per
                 * confirm step on a word every workgroup shares */
                if (lane == 0 && cl.nrec)
                    atomicAdd(&P.counters[0], (unsigned long long)cl.nrec);
            }
        }
        if ((P.dbg & 8192) && P.wave_log && lane < 8) {
            /* diagnostic: a confirm wave's entry and end */
            const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
            P.wave_log[((size_t)blockIdx.x * LIT_WAVES + wave) * 8 + lane] =
                lane == 0 ? t_entry : lane == 1 ? t_end : lane == 2 ? 1ull
                : lane == 3 ? dg[0] : lane == 4 ? dg[1] : lane == 5 ? dg[2] : 0ull;
        }
        goto finish; /* the fused finish: one inlined copy for every wave */
    }
    { /* the scanning waves */

    u32 bucket_mask = 0;
    if (!(P.dbg & 2)) {
        u32 present = 0;
        for (int b = 0; b < 16; b++) {
            if (P.conf_off[b]) present |= 1u << b;
        }
        if (T::LB == 8) {
            u32 m8 = present & 0xff;
            bucket_mask = m8 | (m8 << 8) | (m8 << 16) | (m8 << 24);
        } else {
            bucket_mask = (present & 0xffff) | (present << 16);
        }
    }
    LitShared L;
    L.tab = tab;
    L.tab_lds = (u32)(uintptr_t)(lds_u8_t *)smem;
    L.tsel = TEDDY_TAB_LDS | ((lane & 31) << (MODE == VSA_MODE_TEDDY ? 2 : 3));
    L.ring = rings + (size_t)wave * P.qcap * REW;
    L.slots = slots;
    L.tail = &q_tails[wave];
    L.head = &q_heads[wave];
    L.lg = 31 - __clz(P.qcap);
    L.dbg = P.dbg;
    L.diag = diag_lds;

    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    u32 n_seg = 0, n_iter = 0; /* diagnostic (wave_log) */
    if ((P.dbg & 2048) && lane == 0) /* diagnostic: first scanning-wave start */
        atomicMax(&P.counters[8], ~t_start);
    u32 ncand_total = 0;
    u32 ring_tail_cache = 0, ring_head = 0;
    /* scanner expansion's batch (IterState xs / xn), carried across blocks
     * and segments, flushed before the wave ends */
    u32 xp_s[4] = {0, 0, 0, 0}, xp_n = 0;

    /* Segment scheduling: workgroup b owns the host-built list [wg_seg[b],
     * wg_seg[b + 1]) -- an equal share of the bytes (runtime.hip build_plan)
     * -- and its scanning waves take the next segment from an LDS counter:
     * no global atomics in the sweep (dynamic tickets measured 50 us of
     * contention at 32 MiB and ~0.15 us of CU time per segment at 4 GiB,
     * profiles/r04c_launch_sweep.jsonl; and a returning global atomic in
     * the sweep loop made the compiler wait for every chunk in flight,
     * vmcnt(0), at each group start).  The CU's waves, whose issue rates
     * differ ~3x by age, balance by stealing sweep groups from each other
     * (below), so a large block is cut into one segment per wave; without
     * stealing (VSA_STEAL=0) the list's segments shrink toward its end
     * instead (guided sizes). */
    /* the next ticket is taken (lane 0, LDS atomic) during the last group of
     * the current segment's sweep, so its latency hides behind that group
     * without one wave holding a whole segment ahead */
    auto take = [&]() -> u32 {
        u32 t = 0;
        if (lane == 0)
            t = __hip_atomic_fetch_add(&wg_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return t;
    };
    auto resolve = [&](u32 t0) -> u32 {
        const u32 t = readlane_u32(t0, 0);
        /* reloaded per segment (scalar loads) rather than held: the sweep
         * needs the SGPRs */
        const u32 wg_lo = readfirstlane_u32(P.dyn_kib ? dyn_s[0] : P.wg_seg[blockIdx.x]);
        const u32 wg_hi = readfirstlane_u32(P.dyn_kib ? dyn_s[1] : P.wg_seg[blockIdx.x + 1]);
        return wg_lo + t < wg_hi ? wg_lo + t : (u32)P.nsegs;
    };
    /* Work stealing inside the workgroup (P.steal): a wave whose
     * list is exhausted takes the back half of the unclaimed sweep groups of
     * the scanning wave with the most left (one LDS compare-and-swap on the
     * victim's rng word; the victim claims each next group with an LDS
     * atomic add one group ahead, so a group is never both's).  The thief
     * scans [mid, end) as a range of the same segment: its own prologue at
     * the range start, and the segment's last checked iterations when its
     * range reaches the segment end.  Only parts of one block (not packed
     * groups or runs) are stolen. */
    const bool steal_on = P.steal != 0;
    auto steal = [&](u32 &sg, u32 &gs, u32 &ge) -> bool {
        for (int tries = 0; tries < 64; tries++) {
            unsigned long long w = 0;
            if (lane < NS) w = rng[lane];
            const u32 c = (u32)w & 0xfffffu, e = (u32)(w >> 20) & 0xfffffu;
            /* a victim's unclaimed groups count by its issue age (younger
             * waves issue slower: x1 / 1.25 / 1.5 / 2.25 for waves 0-3 / 4-7
             * / 8-11 / 12+, quarter units; the per-wave rates of
             * profiles/r04e_waves_4g.txt), and the thief takes the share that
             * would end both together.  Measured against equal weights
             * (profiles/r04m_sweep.jsonl, kernel us, twice each): 4 GiB 850 /
             * 848 against 864 / 857, 1 GiB 242 / 241 against 244 / 246 */
            const u32 wt = lane < 4 ? 4u : lane < 8 ? 5u : lane < 12 ? 6u : 9u;
            u32 best = e > c ? (e - c) * wt : 0u;
            const u32 mine = best;
#pragma unroll
            for (int dd = 32; dd >= 1; dd >>= 1) {
                const u32 o = shfl_xor_u32(best, dd);
                best = o > best ? o : best;
            }
            best = readfirstlane_u32(best);
            if (best < 4u * P.steal) return false;
            const u64 mk = __ballot(mine == best);
            const u32 v = (u32)__ffsll((long long)mk) - 1;
            const unsigned long long wv =
                ((unsigned long long)readlane_u32((u32)(w >> 32), (int)v) << 32) |
                readlane_u32((u32)w, (int)v);
            const u32 vc = (u32)wv & 0xfffffu, ve = (u32)(wv >> 20) & 0xfffffu;
            const u32 wv_ = v < 4 ? 4u : v < 8 ? 5u : v < 12 ? 6u : 9u;
            const u32 wt_ = wave < 4 ? 4u : wave < 8 ? 5u : wave < 12 ? 6u : 9u;
            u32 mid = ve - ((ve - vc) * wv_ + (wv_ + wt_) / 2) / (wv_ + wt_);
            mid = mid < ve ? mid : ve - 1; /* the thief takes at least one */
            const unsigned long long nw = (wv & ~(0xfffffULL << 20)) | ((unsigned long long)mid << 20);
            unsigned long long old = wv;
            if (lane == 0)
                __hip_atomic_compare_exchange_strong(&rng[v], &old, nw, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            old = ((unsigned long long)readlane_u32((u32)(old >> 32), 0) << 32) |
                  readlane_u32((u32)old, 0);
            if (old == wv) {
                sg = (u32)(wv >> 40);
                gs = mid;
                ge = ve;
                return true;
            }
        }
        return false;
    };
    /* segment indices are 32-bit (the plan's descriptors; the kernel's
     * SGPRs are scarce) */
    u32 seg = resolve(take());
    u32 st_gs = 0, st_ge = 0; /* a stolen range: sweep groups [st_gs, st_ge) */
    bool from_list = true;     /* seg came from the workgroup's list */
    for (;;) {
        bool stolen = false;
        if (seg >= P.nsegs) {
            /* out of list work: help the workgroup's waves */
            from_list = false;
            if (steal_on && steal(seg, st_gs, st_ge)) stolen = true;
            else break;
        }
        u32 t_next = 0;
        bool have_next = false;
        bool lastb = true;
        auto prefetch_ticket = [&]() {
            if (!have_next && lastb) {
                t_next = take();
                have_next = true;
            }
        };
        /* the segment's descriptor (runtime.hip build_plan): its blocks,
         * first block | count << 24 (count 0: a part of one block, else
         * `count` whole consecutive blocks), and for a part its offset and
         * length in KiB from the block's origin */
        /* scalar loads (seg is wave-uniform; the plan's tables are written
         * by the host before the launch and only read here) */
        typedef const __attribute__((address_space(4))) u32 cu32;
        const u32 segu = readfirstlane_u32(seg);
        const u32 sbv = ((cu32 *)P.seg_desc)[4 * (size_t)segu];
        u32 d_off = ((cu32 *)P.seg_desc)[4 * (size_t)segu + 1];
        u32 d_len = ((cu32 *)P.seg_desc)[4 * (size_t)segu + 2];
        if (P.dyn_kib) {
            /* dynamic shares: the part of the segment (a part of one block)
             * inside this workgroup's KiB range */
            const u32 d_pos = ((cu32 *)P.seg_desc)[4 * (size_t)segu + 3];
            const u32 lk = readfirstlane_u32(dyn_s[2]), hk = readfirstlane_u32(dyn_s[3]);
            const u32 a = d_pos > lk ? d_pos : lk;
            const u32 e = d_pos + d_len < hk ? d_pos + d_len : hk;
            d_off += a - d_pos;
            d_len = e > a ? e - a : 0u;
        }
        const u32 gcount = sbv >> 24;
        /* a run (VSA_BLK_RUN, FDR / Teddy): the segment's back-to-back
         * blocks are one range -- one prologue, one sweep, two checked
         * iterations -- instead of that per block.  What crosses a block
         * boundary is harmless: a literal inside a block has all its filter
         * fields inside it (a field past the literal's length accepts any
         * byte), so the filter stays a superset, and the confirm drops a
         * literal starting before its block (e + 1 >= size) and keys on
         * bytes of the literal only (fdr_confirm_runtime.h:43-102).  The FDR
         * start state is applied to the run's first block only (it only
         * removes candidates).  The run's block ends sit in two VGPRs (block
         * lane, lane + 64, relative to the run's first byte); S.blk / S.run_nxt
         * follow the sweep, and a pushed chunk names the block of its first
         * byte. */
        const u32 first = sbv & 0xffffffu;
        bool run = false;
        if constexpr (MODE != VSA_MODE_NOOD)
            run = gcount > 1 &&
                  (((cu32 *)P.blocks)[(size_t)first * (sizeof(VsaBlock) / 4) +
                                      offsetof(VsaBlock, flags) / 4] & VSA_BLK_RUN);
        u32 rend0 = 0xffffffffu, rend1 = 0xffffffffu;
        const u32 nblk = run ? 1u : (gcount ? gcount : 1u);
        for (u32 gi = 0; gi < nblk; gi++) {
        lastb = gi + 1 == nblk;
        const u32 blk = first + gi;
        const VsaBlock B = load_block(P.blocks, blk);
        SegCtx S;
        S.blk = blk;
        S.blo = (int64_t)B.base + mis;
        S.bhi = S.blo + (int64_t)B.len;
        S.run_nxt = INT64_MAX;
        u32 rb = 0; /* runs: index of block S.blk in the run */
        if (run) {
            if (lane < gcount) {
                const VsaBlock &bl = P.blocks[first + lane];
                rend0 = (u32)(bl.base + bl.len - B.base);
            }
            if (lane + 64 < gcount) {
                const VsaBlock &bl = P.blocks[first + 64 + lane];
                rend1 = (u32)(bl.base + bl.len - B.base);
            }
            S.bhi = S.blo + (int64_t)(gcount > 64 ? readlane_u32(rend1, gcount - 65)
                                                  : readlane_u32(rend0, gcount - 1));
            S.run_nxt = S.blo + (int64_t)readlane_u32(rend0, 0);
        }
        /* runs: after the iteration at ib, move to the next block once the
         * sweep has reached it (blocks >= 1 KiB: at most one per iteration) */
        /* the next block start as a 32-bit offset from the run's first byte
         * (a run spans one segment), so the per-iteration test is a scalar
         * compare, not a 64-bit vector one */
        int32_t rn32 = run ? (int32_t)readlane_u32(rend0, 0) : INT32_MAX;
        auto run_adv = [&](int64_t ib) {
            if ((int32_t)(ib - S.blo) + 1024 >= rn32) {
                rb++;
                S.blk++;
                const bool last = rb + 1 >= gcount;
                const u32 nx = rb < 64 ? readlane_u32(rend0, rb) : readlane_u32(rend1, rb - 64);
                S.run_nxt = last ? INT64_MAX : S.blo + (int64_t)nx;
                rn32 = last ? INT32_MAX : (int32_t)nx;
            }
        };
        S.vlo = S.blo - (int64_t)B.hist;
        S.stream = (B.flags & VSA_BLK_STREAM) != 0;
        S.qlo = 0;
        if (S.stream) {
            const int64_t back = (MODE == VSA_MODE_NOOD) ? (int64_t)P.nood_len - 1
                                                         : (int64_t)(T::NL - 1);
            if (MODE != VSA_MODE_NOOD || B.start == 0)
                S.qlo = -min((int64_t)B.hlen, back);
        }
        S.start = (int64_t)B.start;
        S.len = S.bhi - S.blo;
        S.zbase = B.zbase;
        S.rlo = B.rlo > S.start ? B.rlo : S.start;
        const int64_t s_lo = (gcount || run) ? B.org : B.org + ((int64_t)d_off << 10);
        const int64_t s_hi =
            (!gcount && s_lo + ((int64_t)d_len << 10) < S.bhi) ? s_lo + ((int64_t)d_len << 10) : S.bhi;
        const u32 niters = (u32)((s_hi - s_lo + 1023) >> 10);
        const int64_t zlo = MODE == VSA_MODE_FDR4 ? B.zbase : S.qlo;

        /* iterations [f0, f1) are interior ("fast"): no byte of the 1 KiB
         * chunk or its successor byte lies outside the block, and the FDR
         * start state / `start` cut-off are behind it.  The rest (at most a
         * couple per block) run the checked path one at a time. */
        const int64_t fast_lo = S.blo + S.rlo + 16;
        u32 f0 = 0, f1 = niters;
        if (s_lo < fast_lo) f0 = (u32)min((int64_t)niters, (fast_lo - s_lo + 1023) >> 10);
        {
            /* need ib + 1024 < bhi  <=>  it < (bhi - s_lo - 1024 + 1023) / 1024 rounded */
            int64_t lim = S.bhi - s_lo - 1024; /* ib - s_lo must be < lim */
            int64_t nf = lim <= 0 ? 0 : (lim + 1023) >> 10;
            if (nf < (int64_t)f1) f1 = (u32)nf;
        }
        if (f1 < f0) f1 = f0;
        const u32 nf = f1 - f0;
        const int64_t fb = s_lo + 1024 * (int64_t)f0;
        uint4 ring[LIT_DEPTH];
        /* The range's first loads are issued together: the prologue bytes,
         * the first checked iteration's chunk (ring[0]) and, when there is
         * no sweep, the last checked iteration's chunk (ring[1]), so a small
         * block costs one memory round trip before its first lookup, not
         * one per step (hsbench corpora).  The sweep's chunks follow the
         * first checked iteration (issuing them earlier keeps 16 more VGPRs
         * live through it and spills). */
        const u32 ng = nf / LIT_DEPTH;
        /* a stolen range starts at sweep group st_gs: its prologue is there,
         * and the owner's first checked iterations are not its own */
        const u32 gs = stolen ? st_gs : 0u;
        const u32 it0 = gs * LIT_DEPTH;
        const int64_t pro_lo = stolen ? fb + 1024 * (int64_t)it0 : s_lo;
        const bool pro1 = lane < (u32)(T::NL - 1);
        const int64_t pp = pro_lo - (T::NL - 1) + (int64_t)lane;
        const bool pro1_in = pro1 && pp - S.blo >= zlo && pp - S.blo < S.len;
        const u8 *safe = (const u8 *)P.blocks;
        const u8 pb0 = load_byte_masked(A, pp, S.vlo, S.bhi, pro1_in, safe);
        /* FDR4 keys also need the two bytes before each position: issued
         * with the others (one memory round trip for the whole prologue) */
        const bool F4P = MODE == VSA_MODE_FDR4;
        const u8 pm2 = F4P ? load_byte_masked(A, pp - 2, S.vlo, S.bhi, pro1_in, safe) : (u8)0;
        const u8 pm1 = F4P ? load_byte_masked(A, pp - 1, S.vlo, S.bhi, pro1_in, safe) : (u8)0;
        const u32 pbb = load_byte_masked(A, pro_lo - 8 + (int64_t)lane, S.vlo, S.bhi, lane < 8, safe);
        /* a range that starts with the sweep (a segment inside a block, the
         * common case of large blocks): its first LIT_DEPTH chunks go out
         * with the prologue bytes, so a segment start waits for one memory
         * round trip, not two (prologue, then the sweep's first chunk) */
        const bool early = (f0 == 0 || stolen) && nf > 0;
        const u8 *sb = uniform_ptr(A + fb);
        if (early) {
#pragma unroll
            for (int k = 0; k < LIT_DEPTH; k++)
                ring[k] = load_wave_kib(sb, it0 + (u32)k < nf ? 1024u * (it0 + k) : 1024u * it0);
        }
        if (!early) {
            ring[0] = make_uint4(0, 0, 0, 0);
            ring[1] = make_uint4(0, 0, 0, 0);
        }
        if (f0 > 0 && !stolen) {
            ring[0] = load_chunk(A, s_lo + 16 * (int64_t)lane, S.bhi);
        }
        /* the tail's first chunk is preloaded only without a sweep (f1 is
         * then max(f0, ...) and the tail starts right after the f0 loop) */
        const bool tail_pre = nf == 0 && f1 < niters && f1 > 0;
        if (tail_pre) {
            const int64_t ibt = s_lo + 1024 * (int64_t)f1;
            ring[1] = load_chunk(A, ibt + 16 * (int64_t)lane, S.bhi);
        }
        /* prologue 1: table spill from positions s_lo-NL+1 .. s_lo-1 */
        IterState is;
        is.ncand = ncand_total;
        is.tail_cache = ring_tail_cache;
        is.head = ring_head;
#pragma unroll
        for (int k = 0; k < 4; k++) is.xs[k] = xp_s[k];
        is.xn = xp_n;
        {
            S_t x = 0;
            if (pro1_in) {
                u32 key;
                if constexpr (MODE == VSA_MODE_FDR4) key = vsa_fdr4_key(pm2, pm1, pb0);
                else key = pb0;
                x = (S_t)lit_lookup<MODE>(tab, key, lane);
                x >>= T::LB * (pro_lo - pp);
            }
            u64 xv = (u64)x;
#pragma unroll
            for (int dd = 1; dd < 8; dd <<= 1) {
                const u32 lo = shfl_down_u32((u32)xv, dd);
                const u32 hi = shfl_down_u32((u32)(xv >> 32), dd);
                xv |= ((u64)hi << 32) | lo;
            }
            is.carry = ((u64)shfl_u32((u32)(xv >> 32), 0) << 32) | shfl_u32((u32)xv, 0);
            /* prologue 2: the 8 bytes before s_lo (keys of the first ends) */
            u64 pb = (u64)pbb << (8 * (lane & 7));
#pragma unroll
            for (int dd = 1; dd < 8; dd <<= 1) {
                const u32 lo = shfl_down_u32((u32)pb, dd);
                const u32 hi = shfl_down_u32((u32)(pb >> 32), dd);
                pb |= ((u64)hi << 32) | lo;
            }
            is.pbytes = ((u64)shfl_u32((u32)(pb >> 32), 0) << 32) | shfl_u32((u32)pb, 0);
        }
        for (u32 it = 0; it < (stolen ? 0u : f0); it++) {
            const int64_t ib = s_lo + 1024 * (int64_t)it;
            uint4 cur = ring[0];
            if (it > 0) cur = load_chunk(A, ib + 16 * (int64_t)lane, S.bhi);
            is = scan_iter<MODE, true, XP, SPLIT>(P, cl, L, S, mis, ib, cur, is, bucket_mask);
            run_adv(ib);
        }
        bool tail_mine = true; /* a stolen-from range leaves its tail to the thief */
        u32 swept = 0;         /* sweep iterations scanned (diagnostic) */
        if (nf > 0) {
            if constexpr (MODE == VSA_MODE_FDR4) {
                /* sweep_enter: the carry (ends 0..2 of the chunk, U[4]'s form)
                 * and the previous chunk's last dword move to lane 0 of p4 /
                 * p3 (IterState) */
                is.p3 = (u32)(is.pbytes >> 32);
                is.p4 = (u32)is.carry;
            }
            /* main sweep: LIT_DEPTH chunks in flight per wave.  ring[k] is
             * consumed and then refilled in place (no register rotation), so
             * each step waits only for its own chunk, the load issued
             * LIT_DEPTH steps ago.  Every load is unconditional (an
             * out-of-range prefetch re-reads the current chunk) so the wait
             * counters stay exact. */
            /* segment base in SGPRs, 32-bit offsets */
            /* Nothing but the sweep's own chunks in flight when it starts
             * (an early range's were issued with its prologue, long done;
             * otherwise they are issued right below): the compiler's wait
             * bookkeeping then sees the same LIT_DEPTH loads, in the same
             * order, on every way into the loop and waits vmcnt(LIT_DEPTH
             * - 1) per iteration.  Without this it merged the paths into a
             * vmcnt(0) at every group start: each group waited for the load
             * issued just before it. */
            __builtin_amdgcn_s_waitcnt(VMCNT0);
            if (!early) {
#pragma unroll
                for (int k = 0; k < LIT_DEPTH; k++)
                    ring[k] = load_wave_kib(sb, (u32)k < nf ? 1024u * k : 0u);
            }
            /* the groups this wave scans: all (or the stolen [gs, ge));
             * with stealing on, each next group is claimed one group ahead
             * and a thief may lower the end meanwhile */
            u32 g_end = stolen ? st_ge : ng;
            const bool stealable = steal_on && gcount == 0 && !run && g_end > gs + 1;
            if (stealable && lane == 0)
                rng[wave] = ((unsigned long long)seg << 40) | ((unsigned long long)g_end << 20) | (gs + 1);
            for (u32 g = gs; g < g_end; g++) {
                unsigned long long clm = 0;
                if (stealable && lane == 0)
                    clm = __hip_atomic_fetch_add(&rng[wave], 1ULL, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
                if (g + 1 == g_end) prefetch_ticket();
#pragma unroll
                for (int k = 0; k < LIT_DEPTH; k++) {
                    const u32 it = g * LIT_DEPTH + k;
                    const int64_t ib = fb + 1024 * (int64_t)it;
                    is = scan_iter<MODE, false, XP, SPLIT>(P, cl, L, S, mis, ib, ring[k], is, bucket_mask);
                    run_adv(ib);
                    const u32 itn = (it + LIT_DEPTH < nf) ? it + LIT_DEPTH : it;
                    ring[k] = load_wave_kib(sb, 1024u * itn);
                }
                if (stealable) {
                    /* group g + 1 is this wave's only if a thief left it */
                    const u32 oe = (readlane_u32((u32)clm, 0) >> 20) |
                                   ((readlane_u32((u32)(clm >> 32), 0) & 0xffu) << 12);
                    if (g + 1 >= oe) {
                        g_end = g + 1;
                        prefetch_ticket();
                    }
                }
            }
            /* the segment's remaining iterations go to whoever scanned its
             * last group */
            tail_mine = g_end == ng;
            const u32 rem = tail_mine ? nf - ng * LIT_DEPTH : 0u;
            swept = (g_end - gs) * LIT_DEPTH + rem;
#pragma unroll
            for (int k = 0; k < LIT_DEPTH - 1; k++) {
                if ((u32)k < rem) {
                    const u32 it = ng * LIT_DEPTH + k;
                    const int64_t ib = fb + 1024 * (int64_t)it;
                    is = scan_iter<MODE, false, XP, SPLIT>(P, cl, L, S, mis, ib, ring[k], is, bucket_mask);
                    run_adv(ib);
                }
            }
            if constexpr (MODE == VSA_MODE_FDR4) {
                /* sweep_leave: back to the scalar carry / pbytes */
                is.pbytes = ((u64)readlane_u32(is.p3, 0) << 32) | (u32)is.pbytes;
                is.carry = readlane_u32(is.p4, 0);
            }
        }
        prefetch_ticket();
        for (u32 it = f1; tail_mine && it < niters; it++) {
            const int64_t ib = s_lo + 1024 * (int64_t)it;
            uint4 cur = ring[1];
            if (it > f1 || !tail_pre) cur = load_chunk(A, ib + 16 * (int64_t)lane, S.bhi);
            is = scan_iter<MODE, true, XP, SPLIT>(P, cl, L, S, mis, ib, cur, is, bucket_mask);
            run_adv(ib);
        }
        n_iter += (stolen ? 0u : f0) + swept + (tail_mine ? niters - f1 : 0u);
        ncand_total = is.ncand;
        ring_tail_cache = is.tail_cache;
        ring_head = is.head;
#pragma unroll
        for (int k = 0; k < 4; k++) xp_s[k] = is.xs[k];
        xp_n = is.xn;
        } /* blocks of the segment */
        n_seg++;
        /* after a stolen range, the list is known to be exhausted */
        seg = (stolen || !from_list) ? (u32)P.nsegs : resolve(t_next);
    }
    if constexpr (XP) {
        /* the last batch of expanded candidates, before this wave's done */
        IterState fs;
        fs.tail_cache = ring_tail_cache;
        fs.head = ring_head;
#pragma unroll
        for (int k = 0; k < 4; k++) fs.xs[k] = xp_s[k];
        fs.xn = xp_n;
        xp_flush(P, cl, L, fs);
    }
    if ((P.dbg & 4096) && P.wave_log && lane < 8) {
        u32 xcc, hwid;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        const unsigned long long v[8] = {t_start, t_end, n_seg, n_iter, blockIdx.x, wave,
                                         xcc, (P.dbg & 8192) ? t_entry : hwid};
        unsigned long long x = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) x = (u32)k == lane ? v[k] : x;
        P.wave_log[((size_t)blockIdx.x * LIT_WAVES + wave) * 8 + lane] = x;
    }
    if ((P.dbg & 2048) && lane == 0) {
        /* diagnostic: earliest / latest scanning-wave end (100 MHz clock):
         * the schedule's tail */
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        atomicMax(&P.counters[9], ~t);
        atomicMax(&P.counters[10], t);
    }
    /* every push of this wave precedes this (LDS order) */
    if (lane == 0) {
        const u32 prev = __hip_atomic_fetch_add(&q_done, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_WORKGROUP);
        if (VSA_DIAG_ON && (P.dbg & 32768) && prev + 1 == NS) {
            /* every scanning wave's adds precede its q_done add (LDS order) */
            for (int k = 0; k < 3; k++) atomicAdd(&P.counters[13 + k], diag_lds[k]);
        }
        if ((P.dbg & 2048) && prev + 1 == NS) /* diagnostic: earliest CU done */
            atomicMax(&P.counters[11], ~(unsigned long long)__builtin_amdgcn_s_memrealtime());
        if (P.wg_time && prev + 1 == NS) {
            /* the schedule's feedback: when the workgroup's last scanning
             * wave finished, and on which XCD (bits 60..63) */
            u32 xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            __hip_atomic_store(&P.wg_time[blockIdx.x],
                               ((unsigned long long)(xcc & 15u) << 60) |
                                   (__builtin_amdgcn_s_memrealtime() & ((1ULL << 60) - 1)),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (P.counters && lane_id() == 0 && ncand_total) {
        atomicAdd(&P.counters[2], (unsigned long long)ncand_total);
        if (P.fin_keys)
            __hip_atomic_fetch_add(&cl.f_cand, ncand_total, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    } /* the scanning waves */
finish:
    /* not Fat Teddy: at 128 VGPRs its scan has no room for the epilogue's
     * registers (it spills); its launches keep vsa_bin_finish */
    if constexpr (MODE != VSA_MODE_FAT)
        if (P.fin_keys) fused_finish(P, cl, (u32 *)smem); /* every wave of the workgroup */
}

template __global__ void vsa_lit_scan<VSA_MODE_FDR4, false, false>(VsaLitParams);
template __global__ void vsa_lit_scan<VSA_MODE_FDR4, true, false>(VsaLitParams);
template __global__ void vsa_lit_scan<VSA_MODE_FDR4, false, true>(VsaLitParams);
template __global__ void vsa_lit_scan<VSA_MODE_FDR4, true, true>(VsaLitParams);
template __global__ void vsa_lit_scan<VSA_MODE_TEDDY, false, false>(VsaLitParams);
template __global__ void vsa_lit_scan<VSA_MODE_FAT, false, false>(VsaLitParams);
template __global__ void vsa_lit_scan<VSA_MODE_NOOD, false, false>(VsaLitParams);

/* ====================================================== binned sort === */

/* Match records sorted without a library sort (runtime.hip
 * queue_bin_sort): bins = VSA_SORT_BINS ranges of end positions; the scan
 * kernel stages each record (key and id) in its bin as it emits it
 * (confirm_multi), and one vsa_bin_finish launch sorts every bin (<= 64
 * records: a register bitonic sort on the full key) into place.  Keys are
 * unique (end, bucket, LitInfo), so the result equals the full sort. */

/* The last launch of a binned scan: the scan's counters [0, 16) go to
 * host memory (fine-grained, h[1..16]) and then h[0] = seq with a
 * system-scope release, which the host polls instead of queueing a copy
 * and an event; then the scan's counters [0, nzero) are zeroed for the
 * next launch, which therefore needs no memset. */
__device__ __forceinline__ void publish_body(unsigned long long *ctr, unsigned long long *h,
                                             unsigned long long seq, uint32_t nzero,
                                             const uint64_t *keys, const uint32_t *ids,
                                             uint32_t kmax) {
    const u32 t = threadIdx.x;
    unsigned long long v = 0;
    if (t < 16) v = ctr[t];
    /* small results (drop-in calls): up to kmax raw records go along, at
     * h[17 ..] (keys) and (u32 *)(h + 17 + kmax) (ids) */
    if (kmax) {
        const uint64_t n = ctr[0];
        const uint32_t m = n < kmax ? (uint32_t)n : kmax;
        uint32_t *hid = (uint32_t *)(h + 17 + kmax);
        for (uint32_t i = t; i < m; i += 256) {
            h[17 + i] = keys[i];
            hid[i] = ids[i];
        }
    }
    __syncthreads(); /* every read before any zeroing */
    if (t < 16) {
        h[1 + t] = v;
        ctr[nzero + t] = v; /* kept on the device too (vsa_pack) */
    }
    for (u32 i = t; i < nzero; i += 256) ctr[i] = 0;
    /* every storing wave waits for its own stores, then the barrier; lane
     * 0's system-scope release orders the flag after all of them */
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        __threadfence_system();
        __hip_atomic_store(&h[0], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

/* publish_body for one wave (no workgroup barrier): wave 0 of
 * vsa_bin_finish's first workgroup publishes while its other waves sort.
 * COH: the counters and feedback records are read with agent-scope atomic
 * loads -- the fused finish publishes from inside the scan, whose other
 * workgroups (on other XCDs) added them with agent-scope atomics */
template <bool COH = false>
__device__ __forceinline__ void publish_wave(unsigned long long *ctr, unsigned long long *h,
                                             unsigned long long seq, uint32_t nzero,
                                             const unsigned long long *fb = nullptr,
                                             unsigned long long *hfb = nullptr, u32 nfb = 0,
                                             uint64_t *pk = nullptr, uint64_t out_cap = 0) {
    auto ld = [](const unsigned long long *p) -> unsigned long long {
        if constexpr (COH)
            return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            return *p;
    };
    const u32 l = lane_id();
    const unsigned long long v = l < 16 ? ld(&ctr[l]) : 0ULL;
    if (pk && l == 0) {
        /* the packed collective buffer's header (vsa_pack's rule): the
         * count, bit 62 when the records are not final -- the output
         * overflowed or a crowded bin left them to a rescan */
        const unsigned long long ovf = ld(&ctr[VSA_CTR_BIN_OVERFLOW]);
        pk[0] = v | ((v > out_cap || ovf) ? (1ULL << 62) : 0ULL);
    }
    /* the scan's schedule-feedback record (device memory) rides along to
     * the host, before the sequence store releases it */
    for (u32 i = l; i < nfb; i += WAVE) hfb[i] = ld(&fb[i]);
    /* every read above before any zeroing below (one wave: program order
     * and a wait for the loads) */
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (l < 16) {
        h[1 + l] = v;
        ctr[nzero + l] = v; /* kept on the device too (vsa_pack) */
    }
    for (u32 i = l; i < nzero; i += WAVE) ctr[i] = 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (l == 0) {
        __threadfence_system();
        __hip_atomic_store(&h[0], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

/* The fused finish's publish (its last workgroup's wave 0): the counters
 * the host reads -- [0] records, [2] confirm candidates, [12] crowd --
 * from the look-back's totals (the others only under debug flags, read
 * back), to host memory and to the kept copy vsa_pack reads; the packed
 * collective buffer's header; the scan counters zeroed for the next
 * launch; then the sequence word with a system-scope release. */
__device__ __forceinline__ void publish_fused(const VsaLitParams &P, unsigned long long n,
                                              unsigned long long cand, bool crowded) {
    const u32 l = lane_id();
    unsigned long long v = 0;
    if (l == 0) v = n;
    else if (l == 2) v = cand;
    else if (l == VSA_CTR_BIN_OVERFLOW) v = crowded ? 1ULL : 0ULL;
    else if (P.dbg && l < 16)
        v = __hip_atomic_load(&P.counters[l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (P.fin_pk && l == 0)
        P.fin_pk[0] = n | ((n > P.out_cap || crowded) ? (1ULL << 62) : 0ULL);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* debug reads before the zeroing */
    if (l < 16) {
        P.fin_pub[1 + l] = v;
        P.counters[144 + l] = v; /* kept on the device too (vsa_pack) */
    }
    for (u32 i = l; i < 144; i += WAVE) P.counters[i] = 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (l == 0)
        __hip_atomic_store(&P.fin_pub[0], P.fin_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* The fused finish (VsaLitParams.fin_keys): the binned sort done by the
 * scan's own workgroups at their end, instead of a vsa_bin_finish launch
 * behind the scan (one kernel boundary and launch less per step).  The plan
 * (plan.hip plan_fused) gives every workgroup its own local bins over the
 * ends it reports (its segments' hull, disjoint from the others' and in
 * workgroup order), so each record's bin is counted in LDS and every bin
 * holds one workgroup's records only: no record crosses workgroups.  What
 * does cross them is one word per workgroup, its record total tagged with
 * the launch's epoch -- agent-scope atomics, coherent across XCDs without
 * the agent-scope release per workgroup a plain-store hand-off needs
 * (round 3: step 1.42 ms, profiles/r03_sort_fused_trace.csv).
 *   B1  every wave's records staged and counted, its counter adds done (the
 *       barrier's release waits for them);
 *   then every wave loads and sorts its 16 local bins in registers (when
 *   sparse: below), while wave 0 first takes the local bins' prefix and
 *   stores the total to fin_agg[w], then, after its own sort, looks back:
 *   the totals of workgroups 0..w-1 (each dispatched before this one, so it
 *   runs or has run and the wait ends);
 *   B2  every wave writes its records at base + offset.  The last workgroup
 *       publishes (publish_fused): its look-back has every other
 *       workgroup's totals -- records, crowd flag, confirm candidates, two
 *       epoch-tagged words each -- so the count the host reads needs no
 *       further round trip.  (The schedule-feedback records go to host
 *       memory from each workgroup; feedback_update skips an incomplete
 *       one.)
 * A crowded local bin (> VSA_SORT_BIN_MAX) was flagged by the scan: its
 * records are skipped here and the host rescans without bins. */
__device__ __forceinline__ void fused_finish(const VsaLitParams &P, const ConfLds &cl, u32 *sc) {
    __syncthreads();
    const u32 tid = threadIdx.x, wave = tid / WAVE, lane = lane_id();
    const u32 w = blockIdx.x, nb = cl.lb_n;
    u32 *loff = sc;             /* [VSA_LBINS] each local bin's first position */
    u32 *misc = sc + VSA_LBINS; /* [0] the workgroup's first output position, [1] its
                                   records, [2] its crowd, [3..5] the lower ones' crowd
                                   and candidates (the publisher's) */
    static_assert(VSA_LBINS == 4 * WAVE, "one wave scans the local bins, 4 per lane");
    if (wave == 0) {
        u32 c[4], t4 = 0;
        bool crowd = false;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const u32 i = 4 * lane + k;
            const u32 v = i < nb ? cl.lbins[i] : 0u;
            crowd |= v > VSA_SORT_BIN_MAX;
            c[k] = v < VSA_SORT_BIN_MAX ? v : VSA_SORT_BIN_MAX;
            t4 += c[k];
        }
        u32 tot;
        u32 e = wave_excl_scan(t4, &tot);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            loff[4 * lane + k] = e;
            e += c[k];
        }
        const bool cr = wave_any(crowd) || cl.f_bad != 0;
        if (lane == 0) {
            const unsigned long long ep = (unsigned long long)P.fin_epoch << 32;
            __hip_atomic_store(&P.fin_agg[2 * w], ep | (cr ? (1ULL << 31) : 0ULL) | tot,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&P.fin_agg[2 * w + 1], ep | cl.f_cand, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        misc[1] = tot;
        misc[2] = cr;
    }
    /* this wave's bins: [16 wave, 16 wave + 16) of the local bins.  When
     * none holds more than 16 records (sparse records: the common case) they
     * take one register sort of <= 4 passes, done before the look-back; a
     * denser wave sorts after it, 4 bins at a time.  A crowded bin (flagged:
     * the host rescans) leaves the wave's bins unsorted. */
    const u32 lb = 16 * wave;
    const u32 nbw = nb > lb ? (nb - lb < 16 ? nb - lb : 16u) : 0u;
    u32 mmax = 0;
    for (u32 j = 0; j < nbw; j++) mmax = cl.lbins[lb + j] > mmax ? cl.lbins[lb + j] : mmax;
    const bool live = mmax != 0 && mmax <= VSA_SORT_BIN_MAX; /* wave-uniform */
    u32 S = 2;
    while (S < mmax && S < WAVE) S <<= 1;
    const u32 per = WAVE / S;
    const u32 np = (nbw + per - 1) / per; /* passes over the 16 bins */
    const bool early = live && np <= 4;   /* every bin <= 16 records: one round */
    const size_t row0 = (size_t)w * VSA_LBINS + lb;
    Bins4 B0;
    if (early) {
        bins16_load(B0, P.bin_keys, P.bin_ids, row0, &cl.lbins[lb], nbw, S, 0, lane);
        bins4_sort(B0, lane);
    }
    /* a round's records to base + their bin's offset + their rank; which bin
     * and slot each lane holds is recomputed (fewer registers live across
     * the look-back: the keys and ids only) */
    auto put = [&](const Bins4 &B, u32 pass0, u32 base) {
        const u32 j_l = lane / S;
#pragma unroll
        for (u32 p = 0; p < 4; p++) {
            if (p >= B.npass) break; /* wave-uniform */
            const u32 j = (pass0 + p) * per + j_l;
            if (j >= nbw || B.r >= cl.lbins[lb + j]) continue;
            const u64 o = (u64)base + loff[lb + j] + B.r;
            if (o < P.out_cap) {
                P.fin_keys[o] = B.k[p];
                P.fin_ids[o] = B.id[p];
            }
            if (P.fin_pk && o < P.fin_pk_cap) {
                P.fin_pk[1 + o] = B.k[p];
                ((uint32_t *)(P.fin_pk + 1 + P.fin_pk_cap))[o] = B.id[p];
            }
        }
    };
    if (wave == 0) {
        /* a bound on the wait (~1 s; never reached when the lower
         * workgroups run): past it the launch is flagged as crowded, so the
         * host discards its records and rescans without bins, instead of
         * the grid never draining */
        u32 base = 0, polls = 0, crowd_lo = 0;
        unsigned long long cand = 0;
        for (u32 v0 = 0; v0 < w; v0 += WAVE) {
            const u32 v = v0 + lane;
            if (v < w) {
                unsigned long long a = 0, b = 0;
                for (; polls < (1u << 20); polls++) {
                    a = __hip_atomic_load(&P.fin_agg[2 * v], __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
                    b = __hip_atomic_load(&P.fin_agg[2 * v + 1], __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
                    if ((u32)(a >> 32) == P.fin_epoch && (u32)(b >> 32) == P.fin_epoch) break;
                    __builtin_amdgcn_s_sleep(2);
                }
                base += (u32)a & 0x7fffffffu;
                crowd_lo |= (u32)(a >> 31) & 1u;
                cand += (u32)b;
            }
        }
        const bool timeout = wave_any(polls >= (1u << 20));
        if (timeout && lane == 0) flag_crowd(P);
#pragma unroll
        for (int dd = 32; dd >= 1; dd >>= 1) {
            base += shfl_xor_u32(base, dd);
            crowd_lo |= shfl_xor_u32(crowd_lo, dd);
            cand += ((unsigned long long)shfl_xor_u32((u32)(cand >> 32), dd) << 32) |
                    shfl_xor_u32((u32)cand, dd);
        }
        if (lane == 0) {
            misc[0] = base;
            /* the last workgroup: the launch's totals for the publish */
            misc[3] = crowd_lo | (timeout ? 1u : 0u);
            misc[4] = (u32)cand;
            misc[5] = (u32)(cand >> 32);
        }
    }
    __syncthreads();
    const u32 base = misc[0];
    if (early) {
        put(B0, 0, base);
    } else if (live) {
        /* denser bins: rounds of 4 passes after the look-back */
        for (u32 pass0 = 0; pass0 < np; pass0 += 4) {
            Bins4 B;
            bins16_load(B, P.bin_keys, P.bin_ids, row0, &cl.lbins[lb], nbw, S, pass0, lane);
            bins4_sort(B, lane);
            put(B, pass0, base);
        }
    }
    if (w + 1 == gridDim.x && wave == 0) {
        /* every other workgroup's totals are in its look-back: the count,
         * the crowd and the candidates need no further memory round trip */
        const unsigned long long n = (unsigned long long)base + misc[1];
        const bool crowded = misc[2] != 0 || misc[3] != 0;
        const unsigned long long cand =
            (((unsigned long long)misc[5] << 32) | misc[4]) + cl.f_cand;
        publish_fused(P, n, cand, crowded);
    }
}

__global__ void __launch_bounds__(256) vsa_publish(unsigned long long *ctr,
                                                   unsigned long long *h,
                                                   unsigned long long seq, uint32_t nzero,
                                                   const uint64_t *keys, const uint32_t *ids,
                                                   uint32_t kmax) {
    publish_body(ctr, h, seq, nzero, keys, ids, kmax);
}

/* Staged binned sort, the one launch behind a scan (runtime.hip
 * queue_bin_sort): the scan wrote every record into its bin's staging
 * slots (bin_keys / bin_ids, VSA_SORT_BIN_MAX per bin) as it counted it and
 * nowhere else, so no scatter pass is needed: they are read from there.  Workgroup w owns bins [64 w, 64 w + 64): it
 * sums the counts of every earlier bin itself (<= 64 KiB of L2 reads; no
 * hand-off between workgroups, which on this chip costs an agent-scope
 * release per workgroup), scans its own 64 counts, and each of its 16 waves
 * sorts 4 bins in registers -- one bitonic network of S = the next power of
 * two >= the largest of the 4 counts, 64 / S bins per pass -- and writes
 * them to their sorted positions.  It also zeroes the same bins of the other
 * count buffer (the next launch counts there: the buffers alternate, since
 * this launch still reads its own), and workgroup 0 publishes the counters
 * to the host (publish_body) at its start: the count and the overflow flags
 * are final when the scan ends, and everything that reads the sorted records
 * is queued on the stream behind this launch.  A bin past VSA_SORT_BIN_MAX
 * (flagged by the scan) or an output past out_cap makes the host rescan
 * (without bins, or with a larger output). */
#define FIN_BINS 64 /* bins per workgroup (1024 threads, 16 waves x 4) */
__global__ void __launch_bounds__(1024) vsa_bin_finish(const uint32_t *counts, uint32_t *counts_next,
                                                     const uint64_t *skeys, const uint32_t *sids,
                                                     uint64_t *okeys,
                                                     uint32_t *oids,
                                                     uint64_t out_cap, unsigned long long *ctr,
                                                     unsigned long long *h,
                                                     unsigned long long seq,
                                                     const unsigned long long *fb,
                                                     unsigned long long *hfb, uint32_t nfb,
                                                     uint64_t *pk, uint64_t pk_cap) {
    __shared__ u32 red[16], cnt[FIN_BINS], off[FIN_BINS];
    static_assert(VSA_SORT_BINS / 4 <= 4 * 1024, "the prefix is 4 uint4 loads per thread");
    const u32 t = threadIdx.x, wv = t / WAVE, lane = lane_id();
    const u32 b0 = blockIdx.x * FIN_BINS;
    const u32 lb = wv * 4; /* this wave's 4 bins */
    /* Two dependent round trips to memory, not four: every count this
     * workgroup needs -- the 64 it owns, this wave's 4 (read directly, to
     * size its sort), and those of every bin before b0 (the prefix) -- is
     * loaded at once; then each wave loads its bins' records before the
     * prefix is reduced, so those loads are in flight across the reduction
     * and both barriers. */
    /* unconditional loads (clamped indices, masked after), in the order they
     * are used, so the compiler can wait for each by count */
    const uint4 mc = *(const uint4 *)(counts + b0 + lb);
    const u32 c64 = counts[b0 + (t & (FIN_BINS - 1))];
    uint4 pv[4];
#pragma unroll
    for (u32 q = 0; q < 4; q++) {
        const u32 i = t + q * 1024;
        pv[q] = ((const uint4 *)counts)[i < b0 / 4 ? i : 0u];
    }
    /* the records of every bin before b0 (this thread's part) */
    u32 s = 0;
#pragma unroll
    for (u32 q = 0; q < 4; q++)
        if (t + q * 1024 < b0 / 4) s += pv[q].x + pv[q].y + pv[q].z + pv[q].w;
    const u32 m[4] = {mc.x, mc.y, mc.z, mc.w};
    u32 mmax = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) mmax = m[j] > mmax ? m[j] : mmax;
    /* empty, or left to the library sort (a crowd: the host reruns) */
    const bool sorting = mmax != 0 && mmax <= VSA_SORT_BIN_MAX;
    Bins4 B;
    bins4_load(B, skeys, sids, (size_t)(b0 + lb), m, sorting, lane);
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) s += shfl_xor_u32(s, dd);
    if (lane == 0) red[wv] = s;
    if (t < FIN_BINS) {
        cnt[t] = c64;
        counts_next[b0 + t] = 0;
    }
    __syncthreads();
    if (wv == 0) {
        u32 base = 0;
#pragma unroll
        for (int kk = 0; kk < 16; kk++) base += red[kk];
        u32 tot;
        const u32 e = wave_excl_scan(cnt[lane], &tot);
        off[lane] = base + e;
    }
    __syncthreads();
    if (blockIdx.x == 0 && wv == 0) publish_wave(ctr, h, seq, 144u, fb, hfb, nfb, pk, out_cap);
    if (!sorting) return;
    bins4_sort(B, lane);
    /* fused vsa_pack (vsa_scan_plan_pack): the records also go straight into
     * the collective's buffer, no pack launch behind this one */
    const u32 o4[4] = {off[lb], off[lb + 1], off[lb + 2], off[lb + 3]};
    bins4_write(B, o4, okeys, oids, out_cap, pk, pk_cap);
}

/* A binned scan's sorted records packed for a collective, on the device
 * (no host round trip): dst = [header | keys (cap) | ids (cap x u32)], the
 * header = the record count, with bit 62 set when the records are not
 * usable as they are (the scan overflowed its output and will run again,
 * or a crowded bin left them to the library sort); min(count, cap)
 * records follow.  saved = the counters vsa_publish kept. */
__global__ void __launch_bounds__(256) vsa_pack(const unsigned long long *saved, uint64_t out_cap,
                                                const uint64_t *keys, const uint32_t *ids,
                                                uint64_t cap, uint64_t *dst) {
    const uint64_t n = saved[0];
    const bool bad = n > out_cap || saved[VSA_CTR_BIN_OVERFLOW] != 0;
    const uint64_t m = bad ? 0 : (n < cap ? n : cap);
    if (blockIdx.x == 0 && threadIdx.x == 0) dst[0] = n | (bad ? (1ULL << 62) : 0ULL);
    uint32_t *did = (uint32_t *)(dst + 1 + cap);
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m;
         i += (uint64_t)gridDim.x * 256) {
        dst[1 + i] = keys[i];
        did[i] = ids[i];
    }
}

/* ======================================================= class scan === */

/* Membership via an 8-dword class bitmap (LDS, 8 banks, broadcast reads).
 * Output: one bit per input byte, 16 bits per lane, stored as u16 (64 lanes
 * write 128 contiguous bytes). */
__global__ void __launch_bounds__(256) vsa_class_scan(VsaClassParams P) {
    __shared__ u32 cls[8], cls2[8];
    const u32 tid = threadIdx.x;
    if (tid < 8) {
        cls[tid] = P.cls[tid];
        cls2[tid] = P.cls2[tid];
    }
    __syncthreads();
    const u32 lane = lane_id();
    const u64 nchunks = (P.len + 15) / 16;
    const u64 stride = (u64)gridDim.x * blockDim.x;
    unsigned long long first = ~0ULL, last = 0, cnt = 0;
    /* data is required 16-byte aligned by the host wrapper */
    for (u64 ci = (u64)blockIdx.x * blockDim.x + tid; ci < ((nchunks + 63) / 64) * 64;
         ci += stride) {
        u32 d[4] = {0, 0, 0, 0};
        u64 p0 = ci * 16;
        bool live = ci < nchunks;
        if (live) {
            if (p0 + 16 <= P.len) {
                uint4 v = *(const uint4 *)(P.data + p0);
                d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
            } else {
                for (u64 k = 0; p0 + k < P.len; k++) {
                    d[k >> 2] |= (u32)P.data[p0 + k] << (8 * (k & 3));
                }
            }
        }
        u32 bits = 0, bits2 = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            u32 ch = (d[j >> 2] >> (8 * (j & 3))) & 0xff;
            bits |= ((cls[ch >> 5] >> (ch & 31)) & 1u) << j;
            if (P.pair) bits2 |= ((cls2[ch >> 5] >> (ch & 31)) & 1u) << j;
        }
        if (P.pair) {
            /* c1 at i and c2 at i+1: next lane's first c2 bit */
            u32 nb = lane_down1(bits2) & 1u;
            if (lane == WAVE - 1) {
                u64 pn = p0 + 16;
                nb = 0;
                if (pn < P.len) {
                    u32 ch = P.data[pn];
                    nb = (cls2[ch >> 5] >> (ch & 31)) & 1u;
                }
            }
            bits = bits & ((bits2 >> 1) | (nb << 15));
        }
        if (live) {
            u64 rem = P.len - p0;
            if (rem < 16) bits &= (1u << rem) - 1u;
            if (P.pair) {
                /* the last byte has no successor */
                if (rem <= 16) bits &= ~(1u << (rem - 1));
            }
        } else {
            bits = 0;
        }
        if (P.bitmap && live) ((uint16_t *)P.bitmap)[ci] = (uint16_t)bits;
        if (bits) {
            u64 f = p0 + (u64)(__ffs(bits) - 1);
            u64 l = p0 + (u64)(31 - __clz(bits)) + 1;
            if (f < first) first = f;
            if (l > last) last = l;
            cnt += __popc(bits);
        }
    }
    /* wave reductions, one atomic per wave */
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        u32 flo = shfl_down_u32((u32)first, d), fhi = shfl_down_u32((u32)(first >> 32), d);
        u64 of = ((u64)fhi << 32) | flo;
        if (of < first) first = of;
        u32 llo = shfl_down_u32((u32)last, d), lhi = shfl_down_u32((u32)(last >> 32), d);
        u64 ol = ((u64)lhi << 32) | llo;
        if (ol > last) last = ol;
        u32 clo = shfl_down_u32((u32)cnt, d), chi = shfl_down_u32((u32)(cnt >> 32), d);
        cnt += ((u64)chi << 32) | clo;
    }
    if (lane == 0) {
        const u32 sl = 16 * (blockIdx.x % P.slots); /* one 128-B line per slot */
        if (first != ~0ULL) atomicMin(P.first + sl, first);
        if (last) atomicMax(P.last + sl, last);
        if (cnt) atomicAdd(P.count + sl, cnt);
    }
}

/* bitmap words are written as u16 lanes; the host sees little-endian u64 */

/* ===================================================== double shufti === */

/* shuftiDoubleExec (shufti_simd.hpp:195-258, x86/shufti.hpp:49-79): byte i
 * matches when some bucket is set in both n1[b[i]] and n2[b[i+1]], except at
 * the last byte of each 16-byte lane of the block being scanned, where the
 * reference's in-lane byte shift feeds 0 (all buckets) for b[i+1].  The
 * three scan stages (unaligned head block, S-aligned blocks, tail block)
 * place those lane ends differently, so each position is tested once per
 * stage it belongs to and the host takes the first stage with a match. */
__global__ void __launch_bounds__(256) vsa_pair_scan(VsaPairParams P) {
    __shared__ u8 n1[256], n2[256];
    const u32 tid = threadIdx.x;
    n1[tid] = P.n1[tid];
    n2[tid] = P.n2[tid];
    __syncthreads();
    const int64_t len = (int64_t)P.len, S = P.vsize, mis = P.mis % P.vsize;
    /* stage geometry (shuftiDoubleExecReal) */
    const bool longbuf = len >= S;
    const bool head = longbuf && mis != 0;
    const int64_t d0 = longbuf ? (mis ? S - mis : 0) : 0;
    const int64_t d_end = longbuf ? d0 + ((len - d0) / S) * S : 0;
    const bool tail = (longbuf ? d_end : 0) != len;
    const int64_t t0 = longbuf ? len - S : 0; /* tail block start */
    unsigned long long fh = ~0ULL, fa = ~0ULL, ft = ~0ULL;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + tid; i < len; i += stride) {
        const u8 a = n1[P.data[i]];
        if (!a) continue;
        const u8 nb = (i + 1 < len) ? n2[P.data[i + 1]] : n2[0];
        if (head && i < S) {
            if ((((i & 15) == 15) ? a : (a & nb)) && (u64)i < fh) fh = (u64)i;
        }
        if (i >= d0 && i < d_end) {
            if (((((i + mis) & 15) == 15) ? a : (a & nb)) && (u64)i < fa) fa = (u64)i;
        }
        if (tail && i >= t0) {
            if (((((i - t0) & 15) == 15) ? a : (a & nb)) && (u64)i < ft) ft = (u64)i;
        }
    }
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) {
        u64 o = ((u64)shfl_down_u32((u32)(fh >> 32), dd) << 32) | shfl_down_u32((u32)fh, dd);
        if (o < fh) fh = o;
        o = ((u64)shfl_down_u32((u32)(fa >> 32), dd) << 32) | shfl_down_u32((u32)fa, dd);
        if (o < fa) fa = o;
        o = ((u64)shfl_down_u32((u32)(ft >> 32), dd) << 32) | shfl_down_u32((u32)ft, dd);
        if (o < ft) ft = o;
    }
    if (lane_id() == 0) {
        if (fh != ~0ULL) atomicMin(P.first, fh);
        if (fa != ~0ULL) atomicMin(P.first + 16, fa);
        if (ft != ~0ULL) atomicMin(P.first + 32, ft);
    }
}

/* ================================================== class scan (LUT) === */

/* Large-buffer byte-class scan (shufti / truffle / vermicelli reduced to a
 * 256-bit class, as vsa_class_scan).  Each workgroup first expands the class
 * into a 64 KiB LDS table over byte PAIRS, T[w] = member(w & 0xff) |
 * member(w >> 8) << 1, so one LDS byte read classifies two input bytes and
 * its address is one v_mad_u32_u16 of the raw input dword (no per-byte
 * extract / shift / test).  One persistent 1024-thread workgroup per CU;
 * wave g owns the contiguous 1 KiB-aligned span [g * span, (g + 1) * span)
 * and sweeps it with a 4-deep ring of unconditional 1 KiB wave loads (the
 * structure tools/probe_stream.hip measured at 6.6-6.8 TB/s).  Output as
 * vsa_class_scan: 1 bit per byte (u16 per lane), first / last / count. */
template <int H>
__device__ __forceinline__ u32 lut_addr16(u32 w, u32 base) {
    u32 r;
    if constexpr (H == 0)
        asm("v_mad_u32_u16 %0, %1, 1, %2" : "=v"(r) : "v"(w), "s"(base));
    else
        asm("v_mad_u32_u16 %0, %1, 1, %2 op_sel:[1,0,0,0]" : "=v"(r) : "v"(w), "s"(base));
    return r;
}
typedef const __attribute__((address_space(3))) u8 lds_cu8_t;
__device__ __forceinline__ u32 lds_ld8(u32 addr) { return *(lds_cu8_t *)(uintptr_t)addr; }

#define CLS_DEPTH 4
/* One 1024-thread workgroup per CU; workgroup b owns bytes [b wspan, (b + 1)
 * wspan) (wspan a multiple of 4 KiB) and its 16 waves take 4 KiB groups of
 * them from an LDS counter, the next group claimed one group ahead: no carry
 * crosses a chunk here, so any wave can take any group, and waves whose issue
 * rates differ by age (up to ~3x) finish together instead of a young wave's
 * static span setting the end. */
__global__ void __launch_bounds__(1024) vsa_class_scan_lut(VsaClassParams P, u64 wspan) {
    __shared__ __align__(16) u8 T[65536];
    __shared__ u8 mem[256];
    __shared__ u32 gctr;
    const u32 tid = threadIdx.x;
    const u32 lane = lane_id();
    const u32 wave = readfirstlane_u32(tid / WAVE);
    /* the workgroup's range: an equal span */
    const u64 lo = (u64)blockIdx.x * wspan;
    const u64 hi = min(lo + wspan, (u64)P.len);
    /* iterations (1 KiB) of the range, the full ones, and its groups */
    const u32 nit = lo < hi ? (u32)((hi - lo + 1023) >> 10) : 0u;
    const u32 nfull = lo < hi ? (u32)min((u64)nit, ((u64)P.len - lo) >> 10) : 0u;
    const u32 ngr = (nit + CLS_DEPTH - 1) / CLS_DEPTH;
    const u8 *sb = uniform_ptr(P.data + (lo < hi ? lo : 0));
    auto chunk_off = [&](u32 it, u32 fallback) { return 1024u * (it < nfull ? it : fallback); };
    /* the first group (= wave) goes out before the table is built (plain
     * loads stay in flight across the barriers); the second is wave + 16 */
    u32 g = wave, gn = wave + 16;
    uint4 ring[CLS_DEPTH];
#pragma unroll
    for (int k = 0; k < CLS_DEPTH; k++)
        ring[k] = g < ngr && nfull ? load_wave_kib(sb, chunk_off(g * CLS_DEPTH + k, 0))
                                   : make_uint4(0, 0, 0, 0);
    if (tid < 256) mem[tid] = (u8)((P.cls[tid >> 5] >> (tid & 31)) & 1u);
    if (tid == 0) {
        gctr = 32;
    }
    __syncthreads();
    {
        /* dword i holds T[4i .. 4i+3]: low bytes 4i & 0xff .., high byte i >> 6 */
        const u32 *m4 = (const u32 *)mem;
        u32 *T4 = (u32 *)T;
        for (u32 i = tid; i < 16384; i += 1024)
            T4[i] = m4[i & 63] | ((u32)mem[i >> 6] * 0x02020202u);
    }
    __syncthreads();
    const u32 base = readfirstlane_u32((u32)(uintptr_t)(lds_cu8_t *)T);
    unsigned long long first = ~0ULL, last = 0, cnt = 0;
    auto classify = [&](u32 it, const uint4 v, u32 valid_bytes) {
        const u32 dw[4] = {v.x, v.y, v.z, v.w};
        u32 bits = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const u32 r0 = lds_ld8(lut_addr16<0>(dw[k], base));
            const u32 r1 = lds_ld8(lut_addr16<1>(dw[k], base));
            bits |= (r0 | (r1 << 2)) << (4 * k);
        }
        if (valid_bytes < 16) bits &= (1u << valid_bytes) - 1u;
        const u64 p0 = lo + 1024 * (u64)it + 16 * lane;
        if (P.bitmap) ((uint16_t *)P.bitmap)[p0 >> 4] = (uint16_t)bits;
        if (bits) {
            const u64 f = p0 + (u64)(__ffs(bits) - 1);
            const u64 l = p0 + (u64)(31 - __clz(bits)) + 1;
            first = f < first ? f : first;
            last = l > last ? l : last;
            cnt += __popc(bits);
        }
    };
    while (g < ngr) {
        u32 gnn = 0;
        if (lane == 0)
            gnn = __hip_atomic_fetch_add(&gctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
        for (int k = 0; k < CLS_DEPTH; k++) {
            const u32 it = g * CLS_DEPTH + k;
            const uint4 v = ring[k];
            /* the next group's chunk k (past the range: this chunk again) */
            const u32 itn = gn < ngr ? gn * CLS_DEPTH + k : it;
            if (nfull) ring[k] = load_wave_kib(sb, chunk_off(itn, it < nfull ? it : 0));
            if (it < nfull) {
                classify(it, v, 16);
            } else if (it < nit) {
                /* the ragged last iteration (buffer end): bytes past len read as 0 */
                const u64 p0 = lo + 1024 * (u64)it + 16 * lane;
                u32 d[4] = {0, 0, 0, 0};
                u32 nv = 0;
                if (p0 < hi) {
                    nv = (u32)min((u64)16, hi - p0);
                    for (u32 b = 0; b < nv; b++) d[b >> 2] |= (u32)P.data[p0 + b] << (8 * (b & 3));
                }
                if (p0 < hi) classify(it, make_uint4(d[0], d[1], d[2], d[3]), nv);
            }
        }
        g = gn;
        gn = readfirstlane_u32(gnn);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        u32 flo = shfl_down_u32((u32)first, d), fhi = shfl_down_u32((u32)(first >> 32), d);
        u64 of = ((u64)fhi << 32) | flo;
        if (of < first) first = of;
        u32 llo = shfl_down_u32((u32)last, d), lhi = shfl_down_u32((u32)(last >> 32), d);
        u64 ol = ((u64)lhi << 32) | llo;
        if (ol > last) last = ol;
        u32 clo = shfl_down_u32((u32)cnt, d), chi = shfl_down_u32((u32)(cnt >> 32), d);
        cnt += ((u64)chi << 32) | clo;
    }
    if (lane == 0) {
        const u32 sl = 16 * ((blockIdx.x * 16 + wave) % P.slots);
        if (first != ~0ULL) atomicMin(P.first + sl, first);
        if (last) atomicMax(P.last + sl, last);
        if (cnt) atomicAdd(P.count + sl, cnt);
    }
}

/* Read-ceiling probe (bench.py's roofline.peak_measured; not a scan): every
 * byte of [A, A + n) read once with 16-byte non-temporal loads, one 1024-
 * thread workgroup per CU, wave w reading static 64 KiB segments w, w + W, ..
 * through a 4-deep 1 KiB ring -- the fastest of the schedules
 * tools/probe_stream.hip measured (6.6 TB/s).  n is a multiple of 64 KiB
 * (the caller rounds down).  The sink store is data-dependent so the loads
 * are kept; it lands in a scratch word, never in scan state. */
__global__ void __launch_bounds__(1024) vsa_read_probe(const uint8_t *A, u64 n, u32 *sink) {
    typedef u32 v4u __attribute__((ext_vector_type(4)));
    const u32 lane = threadIdx.x & 63;
    const u64 W = (u64)gridDim.x * 16;
    const u64 w = (u64)blockIdx.x * 16 + (threadIdx.x >> 6);
    constexpr u64 SEG = 64 << 10;
    constexpr u32 ITERS = SEG >> 10, DEPTH = 4;
    u32 acc = 0;
    for (u64 sg = w; sg * SEG < n; sg += W) {
        const uint8_t *base = A + sg * SEG + 16 * lane;
        v4u ring[DEPTH];
#pragma unroll
        for (u32 k = 0; k < DEPTH; k++) ring[k] = __builtin_nontemporal_load((const v4u *)(base + 1024 * k));
        for (u32 g = 0; g < ITERS / DEPTH; g++) {
#pragma unroll
            for (u32 k = 0; k < DEPTH; k++) {
                const v4u v = ring[k];
                acc ^= v.x + v.y * 3 + v.z * 5 + v.w * 7;
                const u32 it = g * DEPTH + k + DEPTH;
                ring[k] = __builtin_nontemporal_load((const v4u *)(base + 1024 * (it < ITERS ? it : 0)));
            }
        }
    }
    if (acc == 0x9e3779b9u) sink[threadIdx.x & 15] = acc;
}
