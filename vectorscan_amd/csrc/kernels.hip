/*
 * kernels.hip — MI355X (gfx950) kernels for the Vectorscan literal /
 * char-class prefilter hot path.
 *
 *  vsa_lit_scan<MODE>  FDR (fdr.c:145-333) and Teddy / Fat Teddy
 *                      (teddy.c:921-1066, teddy_avx2.c:395-706): first-stage
 *                      filter + exact confirm (fdr_confirm_runtime.h:43-102)
 *                      in one pass.
 *  vsa_nood_scan       noodle (noodle_engine.cpp:75-134).
 *  vsa_class_scan      shufti / truffle / vermicelli reduced to a 256-bit
 *                      byte class (shufti_simd.hpp:89-280, x86/truffle.hpp,
 *                      vermicelli_simd.cpp) -> 1 bit/byte bitmap + first/last.
 *
 * Work decomposition (all kernels): the batch is a list of blocks (each one
 * hwlmExec call); a block is cut into segments of 2^seg_shift end positions;
 * one wave64 owns one segment at a time (dynamic ticket), sweeping it in
 * 1 KiB iterations: lane l loads 16 bytes at iteration_base + 16 l with one
 * global_load_dwordx4 (fully coalesced), so HBM is read exactly once.
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
#define LIT_WAVES 8
#define LIT_THREADS (LIT_WAVES * WAVE)
#define QCAP 256

typedef uint32_t u32;
typedef uint64_t u64;
typedef uint8_t u8;

__device__ __forceinline__ u32 lane_id() { return __lane_id(); }

__device__ __forceinline__ u32 shfl_u32(u32 v, int src) {
    return (u32)__shfl((int)v, src, WAVE);
}
__device__ __forceinline__ u32 shfl_up_u32(u32 v, unsigned d) {
    return (u32)__shfl_up((int)v, d, WAVE);
}
__device__ __forceinline__ u32 shfl_down_u32(u32 v, unsigned d) {
    return (u32)__shfl_down((int)v, d, WAVE);
}

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

__device__ __forceinline__ u8 load_byte_masked(const u8 *A, int64_t aoff,
                                               int64_t lo, int64_t hi) {
    return (aoff >= lo && aoff < hi) ? A[aoff] : (u8)0;
}

/* ===================================================== literal scan === */

template <int MODE>
struct LitTraits;

template <>
struct LitTraits<VSA_MODE_FDR> {
    static constexpr int LB = 8;   /* bits per lane field (= buckets) */
    static constexpr int NL = 8;   /* lanes (positions looked back) */
    static constexpr int CW = 4;   /* conf dwords for 16 ends */
    static constexpr bool KEY16 = true;
    typedef u64 S_t;
};
template <>
struct LitTraits<VSA_MODE_TEDDY> {
    static constexpr int LB = 8;
    static constexpr int NL = 4;
    static constexpr int CW = 4;
    static constexpr bool KEY16 = false;
    typedef u32 S_t;
};
template <>
struct LitTraits<VSA_MODE_FAT> {
    static constexpr int LB = 16;
    static constexpr int NL = 4;
    static constexpr int CW = 8;
    static constexpr bool KEY16 = false;
    typedef u64 S_t;
};

struct ConfLds {
    u64 andmsk[16];
    u64 mult[16];
    u32 nbits[16];
    u32 off[16];
};

/* Confirm one queued candidate (one per lane).  ent = aoff<<24 | blk<<4 | b */
__device__ __forceinline__ void confirm_entry(const VsaLitParams &P,
                                              const u8 *A, u32 mis, u64 ent,
                                              const ConfLds &cl) {
    u32 b = (u32)(ent & 15);
    u32 blk = (u32)((ent >> 4) & 0xfffff);
    int64_t aoff = (int64_t)(ent >> 24);
    const VsaBlock &B = P.blocks[blk];
    int64_t blo = (int64_t)B.base + mis;
    int64_t e = aoff - blo; /* block-relative end */
    /* 8 bytes ending at e; bytes before the block read as 0 (fdr.c:798) */
    u64 key = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        int64_t p = aoff - 7 + k;
        u64 byte = (p >= blo) ? (u64)A[p] : 0;
        key |= byte << (8 * k);
    }
    u32 off = cl.off[b];
    const u8 *fc = P.conf_base + off;
    u32 nb = cl.nbits[b];
    u32 c = (u32)(((key & cl.andmsk[b]) * cl.mult[b]) >> (64 - nb));
    u32 st = *(const u32 *)(fc + 32 + 4 * (size_t)c);
    if (!st) return;
    const u8 *li = fc + st;
    u8 next;
    do {
        const uint4 w0 = *(const uint4 *)li;       /* v, msk */
        const uint4 w1 = *(const uint4 *)(li + 16); /* groups, id|size|flags|next */
        u64 v = ((u64)w0.y << 32) | w0.x;
        u64 msk = ((u64)w0.w << 32) | w0.z;
        u32 id = w1.z;
        u32 size = w1.w & 0xff;
        next = (u8)(w1.w >> 16);
        if ((key & msk) == v && e + 1 >= (int64_t)size) {
            unsigned long long slot = atomicAdd(&P.counters[0], 1ULL);
            if (slot < P.out_cap) {
                u64 end_abs = (u64)B.base + (u64)e;
                u64 lidx = ((u64)(li - fc) >> 5) & VSA_KEY_LI_MASK;
                P.out_keys[slot] = (end_abs << VSA_KEY_END_SHIFT) |
                                   ((u64)b << VSA_KEY_BUCKET_SHIFT) | lidx;
                P.out_ids[slot] = id;
            }
        }
        li += 32;
    } while (next);
}

template <int MODE>
__device__ __forceinline__ u64 lit_lookup(const void *tab, u32 key, u32 lane) {
    if constexpr (MODE == VSA_MODE_FDR) {
        return ((const u64 *)tab)[key];
    } else if constexpr (MODE == VSA_MODE_TEDDY) {
        return ((const u32 *)tab)[(key << 5) | (lane & 31)];
    } else {
        return ((const u64 *)tab)[(key << 5) | (lane & 31)];
    }
}

/* key for position j (0..15) of the lane's 16-byte chunk d[0..3], nx =
 * byte after the chunk */
template <int MODE>
__device__ __forceinline__ u32 lit_key(const u32 d[5], int j, u32 dmask) {
    if constexpr (LitTraits<MODE>::KEY16) {
        u32 w = (j & 3) ? __builtin_amdgcn_alignbyte(d[(j >> 2) + 1], d[j >> 2], j & 3)
                        : d[j >> 2];
        return w & dmask;
    } else {
        return (d[j >> 2] >> (8 * (j & 3))) & 0xff;
    }
}

/* Process one 1 KiB iteration.  Returns S_out of lane 63 in *carry. */
template <int MODE, bool EDGE>
__device__ __forceinline__ void lit_iter(const VsaLitParams &P, const u8 *A,
                                         u32 mis, const void *tab, u32 blk,
                                         const VsaBlock &B, int64_t ib,
                                         int64_t s_lo, int64_t s_hi,
                                         u64 *carry, u64 *queue, u32 *qn,
                                         const ConfLds &cl, u32 bucket_mask,
                                         u32 d_next[4], bool have_next) {
    typedef LitTraits<MODE> T;
    typedef typename T::S_t S_t;
    const u32 lane = lane_id();
    const int64_t blo = (int64_t)B.base + mis; /* aoff of block byte 0 */
    const int64_t bhi = blo + (int64_t)B.len;
    const int64_t p0 = ib + 16 * (int64_t)lane; /* aoff of lane's first byte */
    const int64_t q0 = p0 - blo;                /* block-relative */

    u32 d[5];
    d[0] = d_next[0];
    d[1] = d_next[1];
    d[2] = d_next[2];
    d[3] = d_next[3];
    (void)have_next;
    /* byte after the chunk: lane+1's first byte; lane 63 loads it */
    u32 nx = shfl_down_u32(d[0], 1);
    if (lane == WAVE - 1) {
        int64_t pn = p0 + 16;
        nx = (pn < bhi) ? (u32)A[pn] : 0u;
    }
    d[4] = nx & 0xff;
    if (EDGE) {
        /* zero bytes outside the block */
#pragma unroll
        for (int w = 0; w < 4; w++) {
            u32 m = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                int64_t p = p0 + 4 * w + k;
                if (p >= blo && p < bhi) m |= 0xffu << (8 * k);
            }
            d[w] &= m;
        }
        if (p0 + 16 < blo || p0 + 16 >= bhi) d[4] = 0;
    }

    /* own contributions: running state over the lane's 16 positions */
    u32 c[T::CW];
#pragma unroll
    for (int i = 0; i < T::CW; i++) c[i] = 0;
    S_t S = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        u32 key = lit_key<MODE>(d, j, P.dmask);
        S_t x = (S_t)lit_lookup<MODE>(tab, key, lane);
        if (EDGE) {
            int64_t q = q0 + j;
            bool valid;
            if constexpr (MODE == VSA_MODE_FDR) {
                valid = q >= B.zbase && q < (int64_t)B.len;
            } else {
                valid = q >= 0 && q < (int64_t)B.len;
            }
            if (!valid) x = 0;
        }
        S |= x;
        if constexpr (T::LB == 8) {
            /* insert low byte of S as byte (j&3) of c[j>>2] */
            const u32 sel = 0x03020100u & ~(0xffu << (8 * (j & 3)));
            c[j >> 2] = __builtin_amdgcn_perm((u32)S, c[j >> 2],
                                              sel | (0x04u << (8 * (j & 3))));
        } else {
            c[j >> 1] |= ((u32)S & 0xffffu) << (16 * (j & 1));
        }
        S >>= T::LB;
    }
    /* spill from the previous lane (lane 0: from the previous iteration) */
    u64 s_out = (u64)S;
    u32 in_lo = shfl_up_u32((u32)s_out, 1);
    u32 in_hi = shfl_up_u32((u32)(s_out >> 32), 1);
    u64 s_in = ((u64)in_hi << 32) | in_lo;
    if (lane == 0) s_in = *carry;
    {
        u32 lo = (u32)shfl_u32((u32)s_out, WAVE - 1);
        u32 hi = (u32)shfl_u32((u32)(s_out >> 32), WAVE - 1);
        *carry = ((u64)hi << 32) | lo;
    }
    c[0] |= (u32)s_in;
    if constexpr (sizeof(S_t) == 8) c[1] |= (u32)(s_in >> 32);

    if (EDGE) {
        if constexpr (MODE == VSA_MODE_FDR) {
            /* start state: byte i applies to end start + i.  The short zone
             * shifts fdr->start by 16 - (len - start) bytes against a scan
             * that begins at len - 16 (fdr.c:372-440, :712-720), which lands
             * it on `start` as well. */
#pragma unroll
            for (int j = 0; j < 16; j++) {
                int64_t r = q0 + j - (int64_t)B.start;
                if (r >= 0 && r < 16) {
                    u64 st = r < 8 ? P.state_lo : P.state_hi;
                    u32 sb = (u32)(st >> (8 * (r & 7))) & 0xff;
                    c[j >> 2] |= sb << (8 * (j & 3));
                }
            }
        }
        /* report only ends in [max(start, s_lo), min(len, s_hi)) */
        int64_t elo = s_lo > (int64_t)B.start ? s_lo : (int64_t)B.start;
        int64_t ehi = s_hi < (int64_t)B.len ? s_hi : (int64_t)B.len;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            int64_t q = q0 + j;
            if (q < elo || q >= ehi) {
                if constexpr (T::LB == 8) c[j >> 2] |= 0xffu << (8 * (j & 3));
                else c[j >> 1] |= 0xffffu << (16 * (j & 1));
            }
        }
    }

    /* candidate bits, empty buckets masked (do_confirm_fdr skips cf == 0) */
    u32 n = 0;
#pragma unroll
    for (int i = 0; i < T::CW; i++) {
        c[i] = ~c[i] & bucket_mask;
        n += __popc(c[i]);
    }
    if (!__any(n != 0)) return;

    u32 total;
    u32 pos = wave_excl_scan(n, &total);
    /* make room: confirm 64 at a time while the queue would overflow */
    while (*qn + total > QCAP) {
        u32 avail = *qn < (u32)WAVE ? *qn : (u32)WAVE;
        if (lane < avail) confirm_entry(P, A, mis, queue[*qn - avail + lane], cl);
        *qn -= avail;
        if (avail == 0) break;
    }
    if (*qn + total <= QCAP) {
        u32 w = *qn + pos;
#pragma unroll
        for (int i = 0; i < T::CW; i++) {
            u32 bits = c[i];
            while (bits) {
                u32 bit = __ffs(bits) - 1;
                bits &= bits - 1;
                u32 jj, bk;
                if constexpr (T::LB == 8) {
                    jj = 4 * i + (bit >> 3);
                    bk = bit & 7;
                } else {
                    jj = 2 * i + (bit >> 4);
                    bk = bit & 15;
                }
                u64 aoff = (u64)(p0 + jj);
                queue[w++] = (aoff << 24) | ((u64)blk << 4) | bk;
            }
        }
        *qn += total;
    } else {
        /* pathological burst (> QCAP candidates in 1 KiB): confirm in place */
#pragma unroll
        for (int i = 0; i < T::CW; i++) {
            u32 bits = c[i];
            while (bits) {
                u32 bit = __ffs(bits) - 1;
                bits &= bits - 1;
                u32 jj, bk;
                if constexpr (T::LB == 8) {
                    jj = 4 * i + (bit >> 3);
                    bk = bit & 7;
                } else {
                    jj = 2 * i + (bit >> 4);
                    bk = bit & 15;
                }
                u64 aoff = (u64)(p0 + jj);
                confirm_entry(P, A, mis, (aoff << 24) | ((u64)blk << 4) | bk, cl);
            }
        }
    }
    /* drain full rounds */
    while (*qn >= (u32)WAVE) {
        confirm_entry(P, A, mis, queue[*qn - WAVE + lane], cl);
        *qn -= WAVE;
    }
}

template <int MODE, bool LDS_TABLE>
__global__ void __launch_bounds__(LIT_THREADS)
vsa_lit_scan(VsaLitParams P) {
    typedef LitTraits<MODE> T;
    extern __shared__ __align__(16) u8 smem[];
    __shared__ ConfLds cl;
    const u32 tid = threadIdx.x;
    const u32 lane = lane_id();
    const u32 wave = tid / WAVE;

    /* table -> LDS */
    u32 tab_bytes = 0;
    const void *tab;
    if constexpr (MODE == VSA_MODE_FDR) {
        if (LDS_TABLE) {
            tab_bytes = P.table_entries * 8;
            const uint4 *src = (const uint4 *)P.table;
            uint4 *dst = (uint4 *)smem;
            for (u32 i = tid; i < tab_bytes / 16; i += LIT_THREADS) dst[i] = src[i];
            tab = smem;
        } else {
            tab = P.table;
        }
    } else if constexpr (MODE == VSA_MODE_TEDDY) {
        tab_bytes = 256 * 32 * 4;
        u32 *dst = (u32 *)smem;
        for (u32 i = tid; i < 256 * 32; i += LIT_THREADS) {
            dst[i] = (u32)P.table[i >> 5];
        }
        tab = smem;
    } else {
        tab_bytes = 256 * 32 * 8;
        u64 *dst = (u64 *)smem;
        for (u32 i = tid; i < 256 * 32; i += LIT_THREADS) dst[i] = P.table[i >> 5];
        tab = smem;
    }
    if (tid < 16) {
        u32 off = P.conf_off[tid];
        cl.off[tid] = off;
        if (off) {
            const u8 *fc = P.conf_base + off;
            cl.andmsk[tid] = *(const u64 *)fc;
            cl.mult[tid] = *(const u64 *)(fc + 8);
            cl.nbits[tid] = *(const u32 *)(fc + 16);
        } else {
            cl.andmsk[tid] = 0;
            cl.mult[tid] = 0;
            cl.nbits[tid] = 1;
        }
    }
    __syncthreads();

    u32 bucket_mask = 0;
    {
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

    u64 *queue = (u64 *)(smem + ((tab_bytes + 15) & ~15u)) + wave * QCAP;
    u32 qn = 0;
    const u32 mis = (u32)((uintptr_t)P.data & 15);
    const u8 *A = P.data - mis;
    const int64_t SEG = (int64_t)1 << P.seg_shift;

    for (;;) {
        unsigned long long t = 0;
        if (lane == 0) t = atomicAdd(&P.counters[1], 1ULL);
        u64 seg = ((u64)shfl_u32((u32)(t >> 32), 0) << 32) | shfl_u32((u32)t, 0);
        if (seg >= P.nsegs) break;
        u32 blk = 0;
        while (blk + 1 < P.nblocks && P.blocks[blk + 1].seg_first <= seg) blk++;
        const VsaBlock B = P.blocks[blk];
        const int64_t blo = (int64_t)B.base + mis;
        const int64_t s_lo = (int64_t)(seg - B.seg_first) * SEG;
        int64_t s_hi = s_lo + SEG;
        if (s_hi > (int64_t)B.len) s_hi = (int64_t)B.len;
        const int64_t zlo = (MODE == VSA_MODE_FDR) ? B.zbase : 0;
        int64_t ib = (blo + s_lo) & ~(int64_t)15;

        /* prologue: spill into the first iteration from positions ib-7..ib-1
         * (lanes 0..6 each look up one position) */
        u64 carry = 0;
        {
            typedef typename T::S_t S_t;
            S_t x = 0;
            if (lane < (u32)(T::NL - 1)) {
                int64_t p = ib - (T::NL - 1) + (int64_t)lane; /* aoff */
                int64_t q = p - blo;
                if (q >= zlo && q < (int64_t)B.len) {
                    u32 key;
                    u8 b0 = load_byte_masked(A, p, blo, blo + (int64_t)B.len);
                    if constexpr (T::KEY16) {
                        u8 b1 = load_byte_masked(A, p + 1, blo, blo + (int64_t)B.len);
                        key = ((u32)b0 | ((u32)b1 << 8)) & P.dmask;
                    } else {
                        key = b0;
                    }
                    x = (S_t)lit_lookup<MODE>(tab, key, lane);
                    x >>= T::LB * (ib - p);
                }
            }
            u64 xv = (u64)x;
#pragma unroll
            for (int d = 1; d < 8; d <<= 1) {
                u32 lo = shfl_down_u32((u32)xv, d);
                u32 hi = shfl_down_u32((u32)(xv >> 32), d);
                xv |= ((u64)hi << 32) | lo;
            }
            carry = ((u64)shfl_u32((u32)(xv >> 32), 0) << 32) | shfl_u32((u32)xv, 0);
        }

        const int64_t it_end = blo + s_hi; /* aoff past the last end */
        u32 dn[4] = {0, 0, 0, 0};
        {
            int64_t p0 = ib + 16 * (int64_t)lane;
            if (p0 < blo + (int64_t)B.len) {
                uint4 v = *(const uint4 *)(A + p0);
                dn[0] = v.x; dn[1] = v.y; dn[2] = v.z; dn[3] = v.w;
            }
        }
        for (; ib < it_end; ib += 16 * WAVE) {
            u32 dc[4] = {dn[0], dn[1], dn[2], dn[3]};
            /* prefetch next iteration */
            {
                int64_t p0n = ib + 16 * WAVE + 16 * (int64_t)lane;
                if (ib + 16 * WAVE < it_end && p0n < blo + (int64_t)B.len) {
                    uint4 v = *(const uint4 *)(A + p0n);
                    dn[0] = v.x; dn[1] = v.y; dn[2] = v.z; dn[3] = v.w;
                }
            }
            /* edge iteration: touches positions outside the fully valid
             * interior, ends outside the segment, or the FDR start state */
            int64_t qa = ib - blo, qb = ib + 16 * WAVE - blo; /* [qa, qb) */
            bool edge = (qa < zlo + 16) || (qa < 0) || (qb + 1 > (int64_t)B.len) ||
                        (qa < s_lo) || (qb > s_hi) || (qa < (int64_t)B.start + 16);
            if (edge) {
                lit_iter<MODE, true>(P, A, mis, tab, blk, B, ib, s_lo, s_hi, &carry,
                                     queue, &qn, cl, bucket_mask, dc, true);
            } else {
                lit_iter<MODE, false>(P, A, mis, tab, blk, B, ib, s_lo, s_hi, &carry,
                                      queue, &qn, cl, bucket_mask, dc, true);
            }
        }
    }
    /* drain the wave's queue */
    while (qn) {
        u32 avail = qn < (u32)WAVE ? qn : (u32)WAVE;
        if (lane < avail) confirm_entry(P, A, mis, queue[qn - avail + lane], cl);
        qn -= avail;
    }
}

template __global__ void vsa_lit_scan<VSA_MODE_FDR, true>(VsaLitParams);
template __global__ void vsa_lit_scan<VSA_MODE_FDR, false>(VsaLitParams);
template __global__ void vsa_lit_scan<VSA_MODE_TEDDY, true>(VsaLitParams);
template __global__ void vsa_lit_scan<VSA_MODE_FAT, true>(VsaLitParams);

/* ========================================================== noodle === */

/* Each lane owns 16 end positions; the 7 bytes before its chunk come from
 * lane-1 (shuffle).  Report e when (u64 of msk_len bytes ending at e & msk)
 * == cmp, with the whole window inside [start, len) (noodle_engine_simd.hpp
 * scanSingleMain/scanDoubleMain bounds). */
__global__ void __launch_bounds__(256) vsa_nood_scan(VsaNoodParams P) {
    const u32 lane = lane_id();
    const u32 mis = (u32)((uintptr_t)P.data & 15);
    const u8 *A = P.data - mis;
    const int64_t SEG = (int64_t)1 << P.seg_shift;
    const u32 ml = P.msk_len;
    for (;;) {
        unsigned long long t = 0;
        if (lane == 0) t = atomicAdd(&P.counters[1], 1ULL);
        u64 seg = ((u64)shfl_u32((u32)(t >> 32), 0) << 32) | shfl_u32((u32)t, 0);
        if (seg >= P.nsegs) break;
        u32 blk = 0;
        while (blk + 1 < P.nblocks && P.blocks[blk + 1].seg_first <= seg) blk++;
        const VsaBlock B = P.blocks[blk];
        const int64_t blo = (int64_t)B.base + mis;
        const int64_t bhi = blo + (int64_t)B.len;
        const int64_t s_lo = (int64_t)(seg - B.seg_first) * SEG;
        int64_t s_hi = s_lo + SEG;
        if (s_hi > (int64_t)B.len) s_hi = (int64_t)B.len;
        int64_t elo = (int64_t)B.start + ml - 1;
        if (elo < s_lo) elo = s_lo;
        for (int64_t ib = (blo + s_lo) & ~(int64_t)15; ib < blo + s_hi; ib += 16 * WAVE) {
            int64_t p0 = ib + 16 * (int64_t)lane;
            u32 d[4] = {0, 0, 0, 0};
            if (p0 < bhi) {
                uint4 v = *(const uint4 *)(A + p0);
                d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
            }
            /* zero bytes outside the block */
            bool edge = (ib < blo) || (ib + 16 * WAVE > bhi);
            if (edge) {
#pragma unroll
                for (int w = 0; w < 4; w++) {
                    u32 m = 0;
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        int64_t p = p0 + 4 * w + k;
                        if (p >= blo && p < bhi) m |= 0xffu << (8 * k);
                    }
                    d[w] &= m;
                }
            }
            u32 pv2 = shfl_up_u32(d[2], 1), pv3 = shfl_up_u32(d[3], 1);
            if (lane == 0) {
                /* 8 bytes before the iteration */
                pv2 = 0; pv3 = 0;
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    u32 b = load_byte_masked(A, p0 - 8 + k, blo, bhi);
                    if (k < 4) pv2 |= b << (8 * k); else pv3 |= b << (8 * (k - 4));
                }
            }
            u32 w[6] = {pv2, pv3, d[0], d[1], d[2], d[3]};
            u32 hits = 0;
#pragma unroll
            for (int j = 0; j < 16; j++) {
                /* 8 bytes ending at p0 + j: bytes [p0+j-7, p0+j] */
                const int bo = 8 + j - 7; /* byte offset in w[] */
                u32 lo, hi;
                if (bo & 3) {
                    lo = __builtin_amdgcn_alignbyte(w[(bo >> 2) + 1], w[bo >> 2], bo & 3);
                    hi = __builtin_amdgcn_alignbyte(w[(bo >> 2) + 2], w[(bo >> 2) + 1], bo & 3);
                } else {
                    lo = w[bo >> 2];
                    hi = w[(bo >> 2) + 1];
                }
                u64 v = (((u64)hi << 32) | lo) >> (8 * (8 - ml));
                if ((v & P.msk) == P.cmp) hits |= 1u << j;
            }
            int64_t q0 = p0 - blo;
#pragma unroll
            for (int j = 0; j < 16; j++) {
                int64_t q = q0 + j;
                if (q < elo || q >= s_hi) hits &= ~(1u << j);
            }
            while (hits) {
                u32 j = __ffs(hits) - 1;
                hits &= hits - 1;
                unsigned long long slot = atomicAdd(&P.counters[0], 1ULL);
                if (slot < P.out_cap) {
                    u64 end_abs = (u64)B.base + (u64)(q0 + j);
                    P.out_keys[slot] = end_abs << VSA_KEY_END_SHIFT;
                    P.out_ids[slot] = P.id;
                }
            }
        }
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
            u32 nb = shfl_down_u32(bits2, 1) & 1u;
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
        if (first != ~0ULL) atomicMin(P.first, first);
        if (last) atomicMax(P.last, last);
        if (cnt) atomicAdd(P.count, cnt);
    }
}

/* bitmap words are written as u16 lanes; the host sees little-endian u64 */
