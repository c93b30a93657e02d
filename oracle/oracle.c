/*
 * oracle.c — TEST INFRASTRUCTURE ONLY.  A scalar CPU restatement of the
 * Vectorscan hot-path runtime, used by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the CHECKER.  Nothing in vectorscan_amd/
 * links, loads or calls this file; the product path is the HIP engine.
 *
 * It reads the same HWLM bytecode the GPU engine reads and reproduces the
 * reference's callback sequence.  Each routine cites what it restates:
 *   hwlmExec              src/hwlm/hwlm.c:178-205 (accel pre-skip :48-105)
 *   noodExec              src/hwlm/noodle_engine.cpp:75-134,
 *                         noodle_engine_simd.hpp:173-273 (scan bounds)
 *   fdrExec               src/fdr/fdr.c:699-825 (zones :362-659,
 *                         get_conf_stride_1/2/4 :145-296, do_confirm :299)
 *   confWithBit           src/fdr/fdr_confirm_runtime.h:43-102
 *   Teddy / Fat Teddy     src/fdr/teddy.c:921-1066 (SSE),
 *                         src/fdr/teddy_avx2.c:395-706 (AVX2 fat),
 *                         teddy_runtime_common.h:146-199, :395-440
 *   shufti / truffle      src/nfa/shufti.cpp:44-71, shufti_simd.hpp:89-280,
 *                         src/nfa/x86/truffle.hpp:36-62
 *   vermicelli            src/nfa/vermicelli_simd.cpp:493-622
 *
 * Parity pin: tests/test_cpu_oracle.py checks every entry point here
 * against the known answers of the reference's own unit tests
 * (unit/internal/{noodle,fdr,shufti,truffle,vermicelli,rvermicelli}.cpp),
 * restated as data in tests/golden/.
 *
 * Flood detection (flood_runtime.h) is restated only as "disabled": the
 * blobs the tests build carry idCount == FDR_FLOOD_MAX_IDS for every char,
 * under which the reference's floodDetect never changes the scan.
 */
#define _GNU_SOURCE 1 /* pthread_setaffinity_np (the harness pinning) */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64a;
typedef unsigned __int128 u128;

#define ROUNDUP_CL(x) (((x) + 63) & ~(size_t)63)

/* --- reference layouts (restated, see vectorscan_amd/csrc/hs_layout.h) -- */
struct o_HWLM {
    u8 type;
    u64a accel1_groups;
    u8 accel1[80] __attribute__((aligned(16)));
    u8 accel0[80] __attribute__((aligned(16)));
};
struct o_nood {
    u32 id;
    u64a msk, cmp;
    u8 msk_len, key_offset, nocase, single, key0, key1;
};
struct o_FDR {
    u32 engineID, size, maxStringLen, numStrings, confOffset, floodOffset;
    u8 stride, domain;
    u16 domainMask;
    u32 tabSize;
    u8 start[16] __attribute__((aligned(16)));
};
struct o_Teddy {
    u32 engineID, size, maxStringLen, numStrings, confOffset, floodOffset;
};
struct o_LitInfo {
    u64a v, msk, groups;
    u32 id;
    u8 size, flags, next;
};
struct o_FDRConfirm {
    u64a andmsk, mult;
    u32 nBits;
    u64a groups;
};

typedef struct {
    u64a end;
    u32 id;
} orc_match;

/* callback emulation: record; return CONTINUE unless told to terminate
 * after `term_after` matches; optional control override */
typedef struct {
    orc_match *out;
    size_t cap;
    size_t n;
    long term_after;
    u64a ret_groups; /* value the emulated callback returns */
    /* digest mode (orc_digest_mt): ends < drop_below are not counted; the
     * rest fold into dsum / dxor as mix64((base + end) << 32 ^ id) */
    int digest;
    u64a drop_below, base, dsum, dxor;
    /* INCLUDED_JUMP emulation (program_runtime.c:2985-2997): after reporting
     * literal id, a Rose program holding squash[id] != 0 clears those
     * buckets from the live FDR confirm word (scratch->fdr_conf, set only
     * during FDR confirms, fdr_confirm_runtime.h:62-64; Teddy passes none,
     * teddy_runtime_common.h:436-439) */
    const u8 *squash;
    size_t squash_n;
} cbctx;

/* splitmix64 finalizer: the per-match term of the order-free match-set
 * digest (count, sum, xor) shared with the GPU-side check in bench.py */
static inline u64a orc_mix64(u64a x) {
    u64a z = x + 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

static u64a emit(cbctx *c, u64a end, u32 id) {
    if (c->digest == 2) {
        /* record mode (orc_records_mt): every end >= drop_below, in callback
         * order, into a growing array */
        if (end >= c->drop_below) {
            if (c->n == c->cap) {
                const size_t nc = c->cap ? 2 * c->cap : 4096;
                orc_match *o = (orc_match *)realloc(c->out, nc * sizeof(orc_match));
                if (!o) return 0; /* terminate: the caller sees the short count */
                c->out = o;
                c->cap = nc;
            }
            c->out[c->n].end = c->base + end;
            c->out[c->n].id = id;
            c->n++;
        }
        return c->ret_groups;
    }
    if (c->digest) {
        if (end >= c->drop_below) {
            const u64a m = orc_mix64(((c->base + end) << 32) ^ id);
            c->dsum += m;
            c->dxor ^= m;
            c->n++;
        }
        return c->ret_groups;
    }
    if (c->n < c->cap) {
        c->out[c->n].end = end;
        c->out[c->n].id = id;
    }
    c->n++;
    if (c->term_after >= 0 && (long)c->n >= c->term_after) {
        return 0; /* HWLM_TERMINATE_MATCHING */
    }
    return c->ret_groups;
}

static inline u8 toupper_c(u8 c) { return (c >= 'a' && c <= 'z') ? c - 0x20 : c; }
static inline int isalpha_c(u8 c) {
    return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z');
}

/* ====================================================== accel engines == */

/* shufti.cpp:44-71: first c with lo[c&15] & hi[c>>4], else buf_end */
long orc_shufti(const u8 *lo, const u8 *hi, const u8 *buf, size_t len) {
    for (size_t i = 0; i < len; i++) {
        u8 c = buf[i];
        if (lo[c & 0xf] & hi[c >> 4]) return (long)i;
    }
    return (long)len;
}

/* rshufti: last member, else -1 (buf - 1) */
long orc_rshufti(const u8 *lo, const u8 *hi, const u8 *buf, size_t len) {
    for (long i = (long)len - 1; i >= 0; i--) {
        u8 c = buf[i];
        if (lo[c & 0xf] & hi[c >> 4]) return i;
    }
    return -1;
}

/* shuftiDoubleExec (shufti_simd.hpp:195-258, x86/shufti.hpp:49-79) with
 * vector width S (VECTORSIZE: 16 SSE, 32 AVX2, 64 AVX-512) and the buffer's
 * address mod S (`mis`).  blockDoubleMask: c = c1 | (c2 shifted down one
 * byte within each 128-bit lane); byte i matches when c != 0xff, i.e. some
 * bucket is clear in both c1[i] and c2[i+1] -- at the last byte of every
 * 16-byte lane the shifted-in c2 is 0, so c1 alone decides there.  Blocks:
 * an unaligned head block at buf (when buf is not S-aligned and len >= S),
 * S-aligned blocks while a whole block fits, then a tail block ending at
 * buf_end (or, when len < S, the buffer zero-padded to S bytes, results
 * >= len dropped).  Returns the first match, or len. */
static long dshufti_block(const u8 *n1, const u8 *n2, const u8 *buf, size_t len, long b0,
                          long S) {
    for (long k = 0; k < S; k++) {
        long i = b0 + k;
        u8 x = (i >= 0 && (size_t)i < len) ? buf[i] : 0;
        u8 m2;
        if ((k & 15) == 15) {
            m2 = 0xff;
        } else {
            long j = i + 1;
            u8 y = (j >= 0 && (size_t)j < len) ? buf[j] : 0;
            m2 = n2[y];
        }
        if (n1[x] & m2) return i;
    }
    return -1;
}

long orc_shufti_double(const u8 *lo1, const u8 *hi1, const u8 *lo2, const u8 *hi2,
                       const u8 *buf, size_t len, long S, long mis) {
    u8 n1[256], n2[256];
    for (int c = 0; c < 256; c++) {
        n1[c] = (u8)~(lo1[c & 15] | hi1[c >> 4]);
        n2[c] = (u8)~(lo2[c & 15] | hi2[c >> 4]);
    }
    long d = 0, r;
    if ((long)len >= S) {
        if (mis % S) {
            if ((r = dshufti_block(n1, n2, buf, len, 0, S)) >= 0) return r;
            d = S - mis % S;
        }
        for (; d + S <= (long)len; d += S) {
            if ((r = dshufti_block(n1, n2, buf, len, d, S)) >= 0) return r;
        }
    }
    if (d != (long)len) {
        if ((long)len < S) {
            r = dshufti_block(n1, n2, buf, len, 0, S);
        } else {
            r = dshufti_block(n1, n2, buf, len, (long)len - S, S);
        }
        if (r >= 0 && r < (long)len) return r;
    }
    return (long)len;
}

/* x86/truffle.hpp:36-62: member iff mask[c>>7][c&15] has bit (c>>4)&7 */
static inline int truffle_member(const u8 *m1, const u8 *m2, u8 c) {
    const u8 *m = (c & 0x80) ? m2 : m1;
    return (m[c & 0xf] >> ((c >> 4) & 7)) & 1;
}

/* Every position's verdict as a bitmap (bit i & 63 of word i >> 6), from
 * the masks (the cfg-2 full-buffer check): shufti_simd.hpp:63-76 /
 * x86/shufti.hpp blockSingleMask (lo[c & 15] & hi[c >> 4] != 0 per byte)
 * and truffle_simd.hpp:56-61 / x86/truffle.hpp blockSingleMask
 * (truffle_member above).  Returns the member count. */
long orc_shufti_bitmap(const u8 *lo, const u8 *hi, const u8 *buf, size_t len, u64a *bits) {
    long n = 0;
    memset(bits, 0, ((len + 63) / 64) * sizeof(u64a));
    for (size_t i = 0; i < len; i++) {
        const u8 c = buf[i];
        if (lo[c & 0xf] & hi[c >> 4]) {
            bits[i >> 6] |= 1ULL << (i & 63);
            n++;
        }
    }
    return n;
}

long orc_truffle_bitmap(const u8 *m1, const u8 *m2, const u8 *buf, size_t len, u64a *bits) {
    long n = 0;
    memset(bits, 0, ((len + 63) / 64) * sizeof(u64a));
    for (size_t i = 0; i < len; i++) {
        if (truffle_member(m1, m2, buf[i])) {
            bits[i >> 6] |= 1ULL << (i & 63);
            n++;
        }
    }
    return n;
}

long orc_truffle(const u8 *m1, const u8 *m2, const u8 *buf, size_t len) {
    for (size_t i = 0; i < len; i++) {
        if (truffle_member(m1, m2, buf[i])) return (long)i;
    }
    return (long)len;
}

long orc_rtruffle(const u8 *m1, const u8 *m2, const u8 *buf, size_t len) {
    for (long i = (long)len - 1; i >= 0; i--) {
        if (truffle_member(m1, m2, buf[i])) return i;
    }
    return -1;
}

/* vermicelli_simd.cpp:493-592 (c must be upper case when nocase) */
long orc_verm(u8 c, int nocase, int negate, int reverse, const u8 *buf,
              size_t len) {
    u8 cm = nocase ? 0xdf : 0xff;
    if (!reverse) {
        for (size_t i = 0; i < len; i++) {
            int eq = (u8)(buf[i] & cm) == c;
            if (eq != negate) return (long)i;
        }
        return (long)len;
    }
    for (long i = (long)len - 1; i >= 0; i--) {
        int eq = (u8)(buf[i] & cm) == c;
        if (eq != negate) return i;
    }
    return -1;
}

/* vermicelliDoubleExecReal :293-358: first i with c1 c2 at i,i+1; else a
 * partial match (last byte == c1) returns len-1; else len. */
long orc_dverm(u8 c1, u8 c2, int nocase, const u8 *buf, size_t len) {
    u8 cm = nocase ? 0xdf : 0xff;
    for (size_t i = 0; i + 1 < len; i++) {
        if ((u8)(buf[i] & cm) == c1 && (u8)(buf[i + 1] & cm) == c2) return (long)i;
    }
    if (len && (u8)(buf[len - 1] & cm) == c1) return (long)len - 1;
    return (long)len;
}

/* vermicelliDoubleMaskedExecReal :425-491 */
long orc_dverm_masked(u8 c1, u8 c2, u8 m1, u8 m2, const u8 *buf, size_t len) {
    for (size_t i = 0; i + 1 < len; i++) {
        if ((u8)(buf[i] & m1) == c1 && (u8)(buf[i + 1] & m2) == c2) return (long)i;
    }
    if (len && (u8)(buf[len - 1] & m1) == c1) return (long)len - 1;
    return (long)len;
}

/* rvermicelliDoubleExecReal :360-423: highest offset of c2 of a pair, i.e.
 * returns i+1 for the last pair (c1 at i, c2 at i+1); a c2 at buf[0] counts
 * as a partial pair.  Returns -1 if none. */
long orc_rdverm(u8 c1, u8 c2, int nocase, const u8 *buf, size_t len) {
    u8 cm = nocase ? 0xdf : 0xff;
    for (long i = (long)len - 1; i >= 1; i--) {
        if ((u8)(buf[i] & cm) == c2 && (u8)(buf[i - 1] & cm) == c1) return i;
    }
    if (len && (u8)(buf[0] & cm) == c2) return 0;
    return -1;
}

/* run_accel accel.c:36-183 on an AccelAux image (accel.h:72-146: type at
 * 0, offset at 1, verm c / dverm c1 c2 m1 m2 at 2.., m128 masks from 16):
 * minimum lengths (16, 17 for the double forms, which stop one byte early),
 * then rv = MAX(c + offset, rv) - offset.  Returns rv - c.  Double shufti
 * is the VECTORSIZE-64 build at the buffer's own alignment. */
long orc_run_accel(const u8 *aux, const u8 *c, size_t len) {
    const u8 type = aux[0], off = aux[1];
    long r;
    switch (type) {
    case 0: /* ACCEL_NONE */
        return 0;
    case 1: /* ACCEL_VERM */
    case 2: /* ACCEL_VERM_NOCASE */
        if (len <= 15) return 0;
        r = orc_verm(aux[2], type == 2, 0, 0, c, len);
        break;
    case 3: /* ACCEL_DVERM */
    case 4: /* ACCEL_DVERM_NOCASE */
        if (len <= 17) return 0;
        r = orc_dverm(aux[2], aux[3], type == 4, c, len - 1);
        break;
    case 17: /* ACCEL_DVERM_MASKED */
        if (len <= 17) return 0;
        r = orc_dverm_masked(aux[2], aux[3], aux[4], aux[5], c, len - 1);
        break;
    case 13: /* ACCEL_SHUFTI */
        if (len <= 15) return 0;
        r = orc_shufti(aux + 16, aux + 32, c, len);
        break;
    case 15: /* ACCEL_TRUFFLE */
        if (len <= 15) return 0;
        r = orc_truffle(aux + 16, aux + 32, c, len);
        break;
    case 14: /* ACCEL_DSHUFTI */
        if (len <= 16) return 0;
        r = orc_shufti_double(aux + 16, aux + 32, aux + 48, aux + 64, c, len - 1, 64,
                              (long)((uintptr_t)c % 64));
        break;
    case 16: /* ACCEL_RED_TAPE */
        r = (long)len;
        break;
    default:
        return 0;
    }
    if (r < (long)off) r = off;
    return r - off;
}

/* ============================================================ noodle == */

/* noodle_engine.cpp:75-134 + scan bounds noodle_engine_simd.hpp:173-273:
 * report end e (ascending) when the msk_len bytes ending at e satisfy
 * (v & msk) == cmp and lie in [start, len). */
static int nood_run(const struct o_nood *n, const u8 *buf, size_t len,
                    size_t start, cbctx *cb) {
    if (len - start < n->msk_len) return 0;
    for (size_t e = start + n->msk_len - 1; e < len; e++) {
        u64a v = 0;
        memcpy(&v, buf + e + 1 - n->msk_len, n->msk_len);
        if ((v & n->msk) != n->cmp) continue;
        if (!emit(cb, e, n->id)) return 1;
    }
    return 0;
}

/* ======================================================= FDR confirm == */

typedef struct {
    const u8 *buf;
    size_t len;
    size_t start;
    cbctx *cb;
    /* streaming (fdrExecStreaming fdr.c:827-855): hend = hbuf + hlen, the
     * 16 bytes before it are readable (garbage before the real history, as
     * the reference guarantees); hlen bounds the confirm overhang */
    const u8 *hend;
    size_t hlen;
    int stream;
    int simd; /* FDR main zone through get_conf_m128 (the SIMD baseline) */
} rtargs;

/* byte at logical position p (0 = buf[0]): history bytes when streaming,
 * the zero fake history (fdr.c:798-806) in block mode, 0 past the end */
static inline u8 rbyte(const rtargs *a, long p) {
    if (p >= 0) return (size_t)p < a->len ? a->buf[p] : 0;
    if (a->stream && p >= -16) return a->hend[p];
    return 0;
}

/* fdr_confirm_runtime.h:43-102 (block mode: len_history == 0) */
static void conf_with_bit(const struct o_FDRConfirm *fc, const rtargs *a,
                          size_t i, u64a *control, u32 *last_match,
                          u64a conf_key, u64a *conf, u32 bit) {
    u32 c = (u32)(((conf_key & fc->andmsk) * fc->mult) >> (64 - fc->nBits));
    const u32 *litIndex = (const u32 *)((const u8 *)fc + 32);
    u32 st = litIndex[c];
    if (!st) return;
    const struct o_LitInfo *li = (const struct o_LitInfo *)((const u8 *)fc + st);
    u8 next;
    do {
        if ((conf_key & li->msk) != li->v) goto out;
        if (*last_match == li->id && (li->flags & 1)) goto out;
        /* overhang into the history beyond len_history (fdr_confirm_runtime.h:79-88) */
        if ((long)i - (long)li->size + 1 < -(long)a->hlen) goto out;
        if (!(li->groups & *control)) goto out;
        *last_match = li->id;
        *control = emit(a->cb, i, li->id);
        if (conf && li->id < a->cb->squash_n && a->cb->squash[li->id]) {
            /* INCLUDED_JUMP: *fdr_conf &= ~squash << (fdr_conf_offset & ~7) */
            *conf &= (~(u64a)a->cb->squash[li->id]) << (bit & ~7u);
        }
    out:
        next = li->next;
        li++;
    } while (next);
}

/* 8 bytes ending at e: history bytes (streaming, fdr.c zone history and
 * teddy_runtime_common.h:395-416 histBytes) or the zero fake history */
static u64a conf_key_at(const rtargs *a, long e) {
    u64a v = 0;
    for (int k = 0; k < 8; k++) v |= (u64a)rbyte(a, e - 7 + k) << (8 * k);
    return v;
}

/* ============================================================== flood == */

/* fdr_internal.h:50-61 */
struct o_FDRFlood {
    u64a allGroups;
    u32 suffix;
    u16 idCount;
    u32 ids[16];
    u64a groups[16];
};

static inline u64a o_ld8(const u8 *p) {
    u64a v;
    memcpy(&v, p, 8);
    return v;
}
/* *(const u64a *)ROUNDUP_PTR(p, 8) */
static inline u64a o_ldr8(const u8 *p) {
    return o_ld8((const u8 *)(((uintptr_t)p + 7) & ~(uintptr_t)7));
}

/* nextFloodDetect flood_runtime.h:41-83 (FLOOD_64): threshold offset */
static size_t o_next_flood_detect(const u8 *buf, size_t len) {
    if (len < 256) return len;
    if (o_ldr8(buf) == o_ldr8(buf + 8)) return 32;
    if (o_ldr8(buf + len / 2) == o_ldr8(buf + len / 2 + 8)) return 32;
    if (o_ldr8(buf + len - 24) == o_ldr8(buf + len - 16)) return 32;
    return len;
}

/* floodDetect flood_runtime.h:85-335 without the reports: at loop pointer
 * i, *fsize = bytes the main loop skips (0: none) and *flp the flood record;
 * returns the next threshold. */
static size_t o_flood_probe(const u8 *buf, size_t len, u32 i, const u8 *fBase, u32 iterBytes,
                            u32 *backoff, u32 *fsize, const struct o_FDRFlood **flp) {
    size_t mainLoopLen = len > 2 * (size_t)iterBytes ? len - 2 * (size_t)iterBytes : 0;
    u32 j = i;
    u8 c = buf[i];
    u32 fIdx = ((const u32 *)fBase)[c];
    const struct o_FDRFlood *fl = (const struct o_FDRFlood *)(fBase + 4 * 256) + fIdx;
    u64a cmpVal = c;
    cmpVal |= cmpVal << 8;
    cmpVal |= cmpVal << 16;
    cmpVal |= cmpVal << 32;
    *fsize = 0;
    *flp = fl;
    if (o_ldr8(buf + i) != cmpVal || fl->idCount >= 16) {
        *backoff *= 2;
        goto floodout;
    }
    if (i < fl->suffix + 7) {
        *backoff *= 2;
        goto floodout;
    }
    j = i - fl->suffix;
    j -= (u32)((uintptr_t)buf + j) & 0x7;
    for (; j + 32 < mainLoopLen; j += 32) {
        if (o_ld8(buf + j + 24) != cmpVal || o_ld8(buf + j + 16) != cmpVal ||
            o_ld8(buf + j + 8) != cmpVal || o_ld8(buf + j) != cmpVal)
            break;
    }
    for (; j + 8 < mainLoopLen; j += 8) {
        if (o_ld8(buf + j) != cmpVal) break;
    }
    for (; j < mainLoopLen; j++) {
        if (buf[j] != c) break;
    }
    if (j > i) {
        j--;
        *fsize = ((j - i) / iterBytes) * iterBytes;
    } else {
        *backoff *= 2;
    }
floodout:
    if ((u32)(j + *backoff) < mainLoopLen - 128) return (size_t)(i > j ? i : j) + *backoff;
    return mainLoopLen;
}

/* the reports of one flood (flood_runtime.h:191-319: the unrolled cases
 * visit ends in groups of 4 (idCount <= 2) or 2, all ids per end) */
static void o_flood_report(const struct o_FDRFlood *fl, u32 i, u32 floodSize, u64a *control,
                           cbctx *cb) {
    if (!fl->idCount || !(*control & fl->allGroups)) return;
    u32 step = fl->idCount <= 2 ? 4 : 2;
    for (u32 t = 0; t < floodSize && (*control & fl->allGroups); t += step) {
        for (u32 k = 0; k < step; k++) {
            for (u32 d = 0; d < fl->idCount; d++) {
                if (*control & fl->groups[d]) *control = emit(cb, i + t + k, fl->ids[d]);
            }
        }
    }
}

/* Teddy build whose loop shape the flood emulation follows (16: SSE
 * teddy.c:1004-1066 with AVX2 Fat Teddy; 32: AVX2 teddy.c:823-888 /
 * teddy_avx2.c:593-660; 64: VBMI teddy.c:335-388 / teddy_avx2.c:395-447) */
static long o_teddy_vsize = 64;
void orc_set_vector_size(long v) { o_teddy_vsize = v; }

/* ================================================================ FDR == */

/* a "zone" buffer as in fdr.c:50-80; we keep a logical byte accessor */
typedef struct {
    const rtargs *a;
    long zstart;   /* logical position of the zone's first scanned byte */
    long zend;     /* logical position one past the last scanned byte */
    u8 shift;
} zone;

/* zones see history before buf (createStartZone / createShortZone copy it,
 * fdr.c:380-560) and a zero post-padding byte */
static inline u8 zbyte(const zone *z, long p) { return rbyte(z->a, p); }

static u128 load_u64_as_u128(const u64a *ft, u32 idx) { return (u128)ft[idx]; }

/* get_conf_stride_{1,2,4} fdr.c:145-296 on a logical zone */
static void get_conf(const zone *z, long it, u32 stride, u16 dmask,
                     const u64a *ft, u64a *conf0, u64a *conf8, u128 *s) {
    u128 st0 = 0, st8 = 0;
    for (int k = 0; k < 8; k += (int)stride) {
        u32 r = ((u32)zbyte(z, it + k) | ((u32)zbyte(z, it + k + 1) << 8)) & dmask;
        st0 |= load_u64_as_u128(ft, r) << (8 * k);
    }
    for (int k = 0; k < 8; k += (int)stride) {
        u32 r = ((u32)zbyte(z, it + 8 + k) | ((u32)zbyte(z, it + 9 + k) << 8)) & dmask;
        st8 |= load_u64_as_u128(ft, r) << (8 * k);
    }
    u128 st = *s | st0;
    *conf0 = ~(u64a)st;
    st >>= 64;
    st |= st8;
    *conf8 = ~(u64a)st;
    *s = st >> 64;
}

/* get_conf_stride_1 fdr.c:145-213 with SSE2 m128 state, as the reference
 * runs it (unaligned 64-bit loads from the buffer, one table load per
 * position, lshiftbyte_m128 = _mm_slli_si128, or-tree, two 8-byte conf
 * words) — the CPU baseline's main-zone loop, where every byte it touches
 * is inside the buffer (the main zone ends 3 bytes before len, fdr.c:649). */
#include <emmintrin.h>

static inline __m128i ld_entry(const u64a *ft, u64a idx) {
    return _mm_loadl_epi64((const __m128i *)(ft + idx));
}

static inline void get_conf_m128(const u8 *itPtr, u64a domain_mask, const u64a *ft,
                                 u64a *conf0, u64a *conf8, __m128i *s) {
    u64a it_hi, it_lo;
    u32 r15;
    memcpy(&it_hi, itPtr, 8);
    memcpy(&it_lo, itPtr + 8, 8);
    memcpy(&r15, itPtr + 15, 4);
    __m128i st0 = ld_entry(ft, domain_mask & it_hi);
    __m128i st1 = _mm_slli_si128(ld_entry(ft, domain_mask & (it_hi >> 8)), 1);
    __m128i st2 = _mm_slli_si128(ld_entry(ft, domain_mask & (it_hi >> 16)), 2);
    __m128i st3 = _mm_slli_si128(ld_entry(ft, domain_mask & (it_hi >> 24)), 3);
    __m128i st4 = _mm_slli_si128(ld_entry(ft, domain_mask & (it_hi >> 32)), 4);
    __m128i st5 = _mm_slli_si128(ld_entry(ft, domain_mask & (it_hi >> 40)), 5);
    __m128i st6 = _mm_slli_si128(ld_entry(ft, domain_mask & (it_hi >> 48)), 6);
    __m128i st7 = _mm_slli_si128(
        ld_entry(ft, domain_mask & ((it_hi >> 56) | (it_lo << 8))), 7);
    __m128i st8 = ld_entry(ft, domain_mask & it_lo);
    __m128i st9 = _mm_slli_si128(ld_entry(ft, domain_mask & (it_lo >> 8)), 1);
    __m128i st10 = _mm_slli_si128(ld_entry(ft, domain_mask & (it_lo >> 16)), 2);
    __m128i st11 = _mm_slli_si128(ld_entry(ft, domain_mask & (it_lo >> 24)), 3);
    __m128i st12 = _mm_slli_si128(ld_entry(ft, domain_mask & (it_lo >> 32)), 4);
    __m128i st13 = _mm_slli_si128(ld_entry(ft, domain_mask & (it_lo >> 40)), 5);
    __m128i st14 = _mm_slli_si128(ld_entry(ft, domain_mask & (it_lo >> 48)), 6);
    __m128i st15 = _mm_slli_si128(ld_entry(ft, domain_mask & r15), 7);
    st0 = _mm_or_si128(_mm_or_si128(_mm_or_si128(st0, st1), _mm_or_si128(st2, st3)),
                       _mm_or_si128(_mm_or_si128(st4, st5), _mm_or_si128(st6, st7)));
    st8 = _mm_or_si128(_mm_or_si128(_mm_or_si128(st8, st9), _mm_or_si128(st10, st11)),
                       _mm_or_si128(_mm_or_si128(st12, st13), _mm_or_si128(st14, st15)));
    __m128i st = _mm_or_si128(*s, st0);
    *conf0 = (u64a)_mm_cvtsi128_si64(st) ^ ~0ULL;
    st = _mm_or_si128(_mm_srli_si128(st, 8), st8);
    *conf8 = (u64a)_mm_cvtsi128_si64(st) ^ ~0ULL;
    *s = _mm_srli_si128(st, 8);
}

static int fdr_run(const struct o_FDR *fdr, const rtargs *a, u64a control) {
    size_t len = a->len, start = a->start;
    if (start >= len) return 0;
    const u64a *ft = (const u64a *)((const u8 *)fdr + ROUNDUP_CL(sizeof(*fdr)));
    const u32 *confBase = (const u32 *)((const u8 *)fdr + fdr->confOffset);
    u32 last_match = ~0U;

    /* prepareZones fdr.c:625-659, in logical coordinates */
    zone zones[3];
    int nz = 0;
    size_t remaining = len - start;
    if (remaining <= 16) {
        zone z = {a, (long)len - 16, (long)len, (u8)(16 - remaining)};
        zones[nz++] = z;
    } else {
        zone zs = {a, (long)start, (long)start + 16, 0};
        zones[nz++] = zs;
        size_t ptr = start + 16;
        size_t main_end = start + ((len - start - 3) / 16) * 16;
        if (main_end > ptr) {
            zone zm = {a, (long)ptr, (long)main_end, 0};
            zones[nz++] = zm;
            ptr = main_end;
        }
        size_t zl = len - ptr;
        size_t first = zl > 16 ? zl - 16 : zl;
        zone ze = {a, (long)len - (long)(zl > 16 ? 32 : 16), (long)len, (u8)(16 - first)};
        zones[nz++] = ze;
    }
    /* getInitState fdr.c:129-142: with history, the table entry of the
     * byte pair before the scan start, moved on one byte; else fdr->start */
    u128 state;
    if (a->hlen) {
        long b = (long)start - 1;
        u32 key = ((u32)rbyte(a, b) | ((u32)rbyte(a, b + 1) << 8)) & fdr->domainMask;
        state = load_u64_as_u128(ft, key) >> 8;
    } else {
        memcpy(&state, fdr->start, 16);
    }
    /* floods: only the main zone's pointer can pass tryFloodDetect (the
     * other zones point floodPtr past their own buffers, fdr.c:392, :509,
     * :569); the skipped iterations leave `state` as it was (FDR_MAIN_LOOP) */
    const u8 *fBase = (const u8 *)fdr + fdr->floodOffset;
    size_t tfd = o_next_flood_detect(a->buf, len);
    u32 backoff = 32;
    for (int zi = 0; zi < nz; zi++) {
        zone *z = &zones[zi];
        const int main_zone = remaining > 16 && zi == 1 && nz == 3;
        /* variable_byte_shift_m128(state, shift) | zone_or_mask[shift] */
        state <<= 8 * z->shift;
        u128 orm = 0;
        for (int k = 0; k < z->shift; k++) orm |= (u128)0xff << (8 * k);
        state |= orm;
        const int fast = a->simd && main_zone && fdr->stride == 1;
        __m128i sv = _mm_setzero_si128();
        if (fast) memcpy(&sv, &state, 16);
        for (long it = z->zstart; it + 16 <= z->zend; it += 16) {
            if (main_zone && (size_t)it > tfd) {
                u32 fsz;
                const struct o_FDRFlood *fl;
                tfd = o_flood_probe(a->buf, len, (u32)it, fBase, 16, &backoff, &fsz, &fl);
                if (fsz) {
                    o_flood_report(fl, (u32)it, fsz, &control, a->cb);
                    it += fsz;
                }
                if (!control) return 1;
            }
            u64a c0, c8;
            if (fast) get_conf_m128(a->buf + it, fdr->domainMask, ft, &c0, &c8, &sv);
            else get_conf(z, it, fdr->stride, fdr->domainMask, ft, &c0, &c8, &state);
            for (int half = 0; half < 2; half++) {
                u64a conf = half ? c8 : c0;
                while (conf) {
                    u32 bit = (u32)__builtin_ctzll(conf);
                    conf &= conf - 1;
                    u32 byte = bit / 8 + 8 * half;
                    u32 b = bit % 8;
                    u32 cf = confBase[b];
                    if (!cf) continue;
                    const struct o_FDRConfirm *fc =
                        (const struct o_FDRConfirm *)((const u8 *)confBase + cf);
                    if (!(fc->groups & control)) continue;
                    long e = it + byte;
                    conf_with_bit(fc, a, (size_t)e, &control, &last_match,
                                  conf_key_at(a, e), &conf, bit);
                }
                if (!control) return 1;
            }
        }
        if (fast) memcpy(&state, &sv, 16);
    }
    return 0;
}

/* ============================================================== Teddy == */

/* FDR_EXEC_TEDDY teddy.c:1004-1066 and FDR_EXEC_FAT_TEDDY teddy_avx2.c:593-
 * 660, restated per 16-byte block.  res[j][i] is the nibble lookup of mask j
 * at byte i (8 or 16 bucket bits); the candidate word for byte i ORs
 * res[j][i - j], taking i - j < 0 from the previous block (palignr with the
 * carried res_old, zero at the start). */
/* The flood checks of one Teddy call: CHECK_FLOOD sits at the top of the
 * main loop (teddy_runtime_common.h:73-80) of the emulated build's shape;
 * events[k] = {loop pointer, bytes skipped, record}.  Returns the count. */
typedef struct {
    u32 i, size;
    const struct o_FDRFlood *fl;
} o_flood_ev;

static size_t o_teddy_floods(const struct o_Teddy *t, const rtargs *a, int fat, u32 nMasks,
                             o_flood_ev *ev, size_t cap) {
    const u8 *buf = a->buf;
    size_t len = a->len, p = a->start, step, iter;
    size_t tfd = o_next_flood_detect(buf, len);
    if (tfd >= len) return 0;
    if (o_teddy_vsize >= 64) {
        /* VBMI: head block of loopBytes = W - (nMasks - 1), then loopBytes */
        step = (fat ? 32 : 64) - (nMasks - 1);
        iter = fat ? 32 : 64;
        if (p + step <= len) p += step;
    } else {
        /* SSE (16-B blocks) / AVX2 (32-B halves; Fat Teddy always 16-B):
         * aligned head block, one block, then two blocks per iteration */
        size_t blk = (!fat && o_teddy_vsize == 32) ? 32 : 16;
        uintptr_t A = (uintptr_t)buf + p;
        uintptr_t ms = (A + blk - 1) & ~(uintptr_t)(blk - 1);
        if (A < ms) p += ms - A;
        if (p + blk <= len) p += blk;
        step = iter = 2 * blk;
    }
    const u8 *fBase = (const u8 *)t + t->floodOffset;
    u32 backoff = 32;
    size_t n = 0;
    for (; p + step <= len; p += step) {
        if (p > tfd) {
            u32 fsz;
            const struct o_FDRFlood *fl;
            tfd = o_flood_probe(buf, len, (u32)p, fBase, (u32)iter, &backoff, &fsz, &fl);
            if (fsz && n < cap) {
                ev[n].i = (u32)p;
                ev[n].size = fsz;
                ev[n].fl = fl;
                n++;
                p += fsz;
            }
        }
    }
    return n;
}

static int teddy_loop(const struct o_Teddy *t, const rtargs *a, u64a control, int fat,
                      u32 nMasks, const o_flood_ev *fev, size_t nfev);

static int teddy_run(const struct o_Teddy *t, const rtargs *a, u64a control,
                     int fat, u32 nMasks) {
    size_t len = a->len;
    /* floods are >= 32 bytes apart; none when the first threshold is len */
    const size_t fcap = o_next_flood_detect(a->buf, len) < len ? len / 32 + 1 : 0;
    o_flood_ev *fev = fcap ? (o_flood_ev *)malloc(fcap * sizeof(o_flood_ev)) : NULL;
    const size_t nfev = fev ? o_teddy_floods(t, a, fat, nMasks, fev, fcap) : 0;
    const int rv = teddy_loop(t, a, control, fat, nMasks, fev, nfev);
    free(fev);
    return rv;
}

static int teddy_loop(const struct o_Teddy *t, const rtargs *a, u64a control, int fat,
                      u32 nMasks, const o_flood_ev *fev, size_t nfev) {
    const u8 *buf = a->buf;
    size_t len = a->len;
    size_t fe = 0;
    long skip_lo = 0, skip_hi = 0;
    const u8 *maskBase = (const u8 *)t + 64;
    const u32 *confBase = (const u32 *)((const u8 *)t + t->confOffset);
    u32 nb = fat ? 16 : 8;
    u32 last_match = ~0U;
    u16 old[4][16];
    memset(old, 0, sizeof(old));

    uintptr_t ptr = (uintptr_t)buf + a->start;
    uintptr_t end = (uintptr_t)buf + len;
    uintptr_t mainStart = (ptr + 15) & ~(uintptr_t)15;
    if (ptr < mainStart) ptr = mainStart - 16;

    for (; ptr < end; ptr += 16) {
        u8 val[16];
        u16 pmask = 0; /* bit i: poison byte i */
        long base = (long)(ptr - (uintptr_t)buf);
        /* vectoredLoad128 teddy_runtime_common.h:146-200: up to
         * min(len_history, nMasks - 1) history bytes before buf */
        long need = (long)(a->hlen < nMasks - 1 ? a->hlen : nMasks - 1);
        for (int i = 0; i < 16; i++) {
            long p = base + i;
            val[i] = (p >= 0 && (size_t)p < len) ? buf[p]
                     : (p < 0 && p >= -need) ? rbyte(a, p) : 0;
            if (p < (long)a->start || (size_t)p >= len) pmask |= (u16)(1u << i);
        }
        u16 res[4][16];
        for (u32 j = 0; j < nMasks; j++) {
            for (int i = 0; i < 16; i++) {
                u8 c = val[i];
                u16 v;
                if (fat) {
                    const u8 *lo = maskBase + j * 64;
                    const u8 *hi = lo + 32;
                    v = (u16)((lo[c & 15] | hi[c >> 4]) |
                              ((lo[16 + (c & 15)] | hi[16 + (c >> 4)]) << 8));
                } else {
                    const u8 *lo = maskBase + j * 32;
                    const u8 *hi = lo + 16;
                    v = (u16)(lo[c & 15] | hi[c >> 4]);
                }
                res[j][i] = v;
            }
        }
        u16 r[16];
        for (int i = 0; i < 16; i++) {
            u16 acc = res[0][i];
            for (u32 j = 1; j < nMasks; j++) {
                acc |= (i >= (int)j) ? res[j][i - j] : old[j][16 + i - j];
            }
            if (pmask & (1u << i)) acc = 0xffff;
            r[i] = acc;
        }
        memcpy(old, res, sizeof(res));
        u16 full = fat ? 0xffff : 0xff;
        for (int i = 0; i < 16; i++) {
            const long e = base + i;
            while (fe < nfev && (long)fev[fe].i <= e) {
                /* the loop pointer passed tryFloodDetect: the flood reports,
                 * then the main loop skips its ends */
                o_flood_report(fev[fe].fl, fev[fe].i, fev[fe].size, &control, a->cb);
                if (!control) return 1;
                skip_lo = fev[fe].i;
                skip_hi = (long)fev[fe].i + fev[fe].size;
                fe++;
            }
            if (e >= skip_lo && e < skip_hi) continue;
            u16 cand = (u16)(~r[i]) & full;
            while (cand) {
                u32 b = (u32)__builtin_ctz(cand);
                cand &= cand - 1;
                u32 cf = confBase[b];
                if (!cf) continue;
                const struct o_FDRConfirm *fc =
                    (const struct o_FDRConfirm *)((const u8 *)confBase + cf);
                if (!(fc->groups & control)) continue;
                conf_with_bit(fc, a, (size_t)e, &control, &last_match,
                              conf_key_at(a, e), NULL, 0);
            }
            if ((i % (fat ? 4 : 8)) == (fat ? 3 : 7) && !control) return 1;
        }
        if (!control) return 1;
        (void)nb;
    }
    return 0;
}

/* ====================================================== entry points == */

static int fdr_dispatch_a(const void *eng, rtargs a, u64a groups) {
    u32 id = *(const u32 *)eng;
    size_t start = a.start;
    if (start >= a.len) return 0;
    if (id == 0) return fdr_run((const struct o_FDR *)eng, &a, groups);
    if (id >= 3 && id <= 10) {
        return teddy_run((const struct o_Teddy *)eng, &a, groups, 1, (id - 3) / 2 + 1);
    }
    if (id >= 11 && id <= 18) {
        return teddy_run((const struct o_Teddy *)eng, &a, groups, 0, (id - 11) / 2 + 1);
    }
    return 2;
}

static int fdr_dispatch_s(const void *eng, const u8 *buf, size_t len, size_t start,
                          u64a groups, cbctx *cb, int simd) {
    rtargs a = {buf, len, start, cb, NULL, 0, 0, simd};
    return fdr_dispatch_a(eng, a, groups);
}

static int fdr_dispatch(const void *eng, const u8 *buf, size_t len,
                        size_t start, u64a groups, cbctx *cb) {
    return fdr_dispatch_s(eng, buf, len, start, groups, cb, 0);
}

/* fdrExec through the SIMD main loop (the CPU baseline engine) */
long orc_fdr_exec_simd(const void *eng, const u8 *buf, size_t len, size_t start,
                       u64a groups, orc_match *out, size_t cap, int *status) {
    cbctx cb = {out, cap, 0, -1, ~0ULL};
    *status = fdr_dispatch_s(eng, buf, len, start, groups, &cb, 1);
    return (long)cb.n;
}

/* fdrExecStreaming fdr.c:827-855 */
long orc_fdr_exec_stream(const void *eng, const u8 *hend, size_t hlen, const u8 *buf,
                         size_t len, size_t start, u64a groups, orc_match *out, size_t cap,
                         long term_after, u64a cb_ret, int *status) {
    cbctx cb = {out, cap, 0, term_after, cb_ret};
    rtargs a = {buf, len, start, &cb, hend, hlen, 1, 0};
    *status = fdr_dispatch_a(eng, a, groups);
    return (long)cb.n;
}

/* noodExecStreaming noodle_engine.cpp:136-185: literals straddling the
 * history (at most msk_len - 1 bytes of each side, scanned byte by byte),
 * then a block scan of buf from 0 */
long orc_nood_exec_stream(const void *eng, const u8 *hend, size_t hlen, const u8 *buf,
                          size_t len, orc_match *out, size_t cap, long term_after,
                          int *status) {
    const struct o_nood *n = (const struct o_nood *)eng;
    cbctx cb = {out, cap, 0, term_after, ~0ULL};
    *status = 0;
    if (len + hlen < n->msk_len) return 0;
    if (hlen && n->msk_len > 1) {
        u8 temp[24]; /* HWLM_LITERAL_MAX_LEN * 2, + slack for the 8-byte loads */
        memset(temp, 0, sizeof(temp));
        size_t tl1 = n->msk_len - 1 < hlen ? n->msk_len - 1 : hlen;
        size_t tl2 = n->msk_len - 1 < len ? n->msk_len - 1 : len;
        memcpy(temp, hend - tl1, tl1);
        memcpy(temp + tl1, buf, tl2);
        for (size_t i = 0; i + n->msk_len <= tl1 + tl2; i++) {
            u64a v;
            memcpy(&v, temp + i, 8);
            if ((v & n->msk) == n->cmp) {
                size_t m_end = i + n->msk_len - 1 - tl1;
                if (!emit(&cb, m_end, n->id)) {
                    *status = 1;
                    return (long)cb.n;
                }
            }
        }
    }
    *status = nood_run(n, buf, len, 0, &cb);
    return (long)cb.n;
}

/* returns number of matches; *status = HWLM_SUCCESS/TERMINATED/ERROR */
long orc_fdr_exec(const void *eng, const u8 *buf, size_t len, size_t start,
                  u64a groups, orc_match *out, size_t cap, long term_after,
                  u64a cb_ret, int *status) {
    cbctx cb = {out, cap, 0, term_after, cb_ret};
    *status = fdr_dispatch(eng, buf, len, start, groups, &cb);
    return (long)cb.n;
}

/* fdrExec with the INCLUDED_JUMP squash table squash[id] (n entries) */
long orc_fdr_exec_squash(const void *eng, const u8 *buf, size_t len, size_t start,
                         u64a groups, orc_match *out, size_t cap, const u8 *squash,
                         size_t squash_n, int *status) {
    cbctx cb = {out, cap, 0, -1, ~0ULL, 0, 0, 0, 0, 0, squash, squash_n};
    *status = fdr_dispatch(eng, buf, len, start, groups, &cb);
    return (long)cb.n;
}

long orc_nood_exec(const void *eng, const u8 *buf, size_t len, size_t start,
                   orc_match *out, size_t cap, long term_after, int *status) {
    cbctx cb = {out, cap, 0, term_after, ~0ULL};
    *status = nood_run((const struct o_nood *)eng, buf, len, start, &cb);
    return (long)cb.n;
}

/* hwlm.c:48-105 accel pre-skip (block mode) */
static size_t accel_block(const u8 *aux, const u8 *buf, size_t len, size_t start) {
    if (len - start < 16) return start;
    u8 type = aux[0], offset = aux[1];
    long r;
    const u8 *p = buf + start;
    size_t n = len - start;
    switch (type) {
    case 1: r = orc_verm(aux[2], 0, 0, 0, p, n); break;
    case 2: r = orc_verm(aux[2], 1, 0, 0, p, n); break;
    case 3: r = orc_dverm(aux[2], aux[3], 0, p, n); break;
    case 4: r = orc_dverm(aux[2], aux[3], 1, p, n); break;
    case 13: r = orc_shufti(aux + 16, aux + 32, p, n); break;
    case 15: r = orc_truffle(aux + 16, aux + 32, p, n); break;
    default: return start;
    }
    long np = (long)start + r;
    if (offset) {
        np -= offset;
        if (np < 0) np = 0;
    }
    return (size_t)np;
}

long orc_hwlm_exec(const void *hwlm, const u8 *buf, size_t len, size_t start,
                   u64a groups, orc_match *out, size_t cap, long term_after,
                   u64a cb_ret, int *status) {
    const struct o_HWLM *h = (const struct o_HWLM *)hwlm;
    const void *eng = (const u8 *)hwlm + ROUNDUP_CL(sizeof(*h));
    cbctx cb = {out, cap, 0, term_after, cb_ret};
    *status = 0;
    if (!groups) return 0;
    if (h->type == 16) {
        *status = nood_run((const struct o_nood *)eng, buf, len, start, &cb);
        return (long)cb.n;
    }
    const u8 *aa = h->accel0;
    if ((groups & ~h->accel1_groups) == 0) aa = h->accel1;
    start = accel_block(aa, buf, len, start);
    *status = fdr_dispatch(eng, buf, len, start, groups, &cb);
    return (long)cb.n;
}

/* run_hwlm_accel hwlm.c:48-80: offset of the accel hit in [p, p + n) */
static size_t hwlm_accel_run(const u8 *aux, const u8 *p, size_t n) {
    switch (aux[0]) {
    case 1: return (size_t)orc_verm(aux[2], 0, 0, 0, p, n);
    case 2: return (size_t)orc_verm(aux[2], 1, 0, 0, p, n);
    case 3: return (size_t)orc_dverm(aux[2], aux[3], 0, p, n);
    case 4: return (size_t)orc_dverm(aux[2], aux[3], 1, p, n);
    case 13: return (size_t)orc_shufti(aux + 16, aux + 32, p, n);
    case 15: return (size_t)orc_truffle(aux + 16, aux + 32, p, n);
    default: return 0;
    }
}

/* do_accel_streaming hwlm.c:114-175 */
static size_t accel_stream(const u8 *aux, const u8 *hbuf, size_t hlen, const u8 *buf,
                           size_t len, size_t start) {
    if (aux[0] == 0 || len - start < 16) return start;
    const u8 offset = aux[1];
    if (!start && hlen) {
        size_t p1 = 0;
        if (hlen >= 16) p1 = hwlm_accel_run(aux, hbuf, hlen);
        int inaccurate = aux[0] == 3 || aux[0] == 4; /* DVERM (nocase) */
        if ((hlen <= 16 || inaccurate) && p1 != hlen && hlen - p1 <= 16) {
            u8 temp[17];
            size_t tlen = hlen - p1;
            memcpy(temp, hbuf + p1, tlen);
            memset(temp + tlen, 0, 17 - tlen);
            if (len) temp[tlen] = buf[0];
            if (hwlm_accel_run(aux, temp, 17) >= tlen) p1 = hlen;
        }
        if (p1 != hlen) return start; /* bailing in history */
    }
    size_t found = start + hwlm_accel_run(aux, buf + start, len - start);
    if (found >= start + offset) start = found - offset;
    return start;
}

/* hwlmExecStreaming hwlm.c:207-247 (hbuf = hend - hlen) */
long orc_hwlm_exec_stream(const void *hwlm, const u8 *hend, size_t hlen, const u8 *buf,
                          size_t len, size_t start, u64a groups, orc_match *out, size_t cap,
                          long term_after, u64a cb_ret, int *status) {
    const struct o_HWLM *h = (const struct o_HWLM *)hwlm;
    const void *eng = (const u8 *)hwlm + ROUNDUP_CL(sizeof(*h));
    *status = 0;
    if (!groups) return 0;
    if (h->type == 16) {
        if (start) {
            cbctx cb = {out, cap, 0, term_after, cb_ret};
            *status = nood_run((const struct o_nood *)eng, buf, len, start, &cb);
            return (long)cb.n;
        }
        return orc_nood_exec_stream(eng, hend, hlen, buf, len, out, cap, term_after, status);
    }
    const u8 *aa = h->accel0;
    if ((groups & ~h->accel1_groups) == 0) aa = h->accel1;
    start = accel_stream(aa, hend - hlen, hlen, buf, len, start);
    return orc_fdr_exec_stream(eng, hend, hlen, buf, len, start, groups, out, cap, term_after,
                               cb_ret, status);
}

/* ====================================== counting helpers (cpu baseline) */

/* Number of FDR first-stage candidates (end, bucket) over a block at stride
 * 1 — a diagnostic for the false-positive rate the confirm stage sees. */
u64a orc_fdr_candidates(const void *eng, const u8 *buf, size_t len) {
    const struct o_FDR *fdr = (const struct o_FDR *)eng;
    const u64a *ft = (const u64a *)((const u8 *)fdr + ROUNDUP_CL(sizeof(*fdr)));
    u64a count = 0;
    for (size_t e = 0; e < len; e++) {
        u64a acc = 0;
        for (int k = 0; k < 8; k++) {
            long p = (long)e - k;
            if (p < 0) break;
            u32 key = ((u32)buf[p] | ((u32)((size_t)(p + 1) < len ? buf[p + 1] : 0) << 8)) &
                      fdr->domainMask;
            acc |= (ft[key] >> (8 * k)) & 0xff;
        }
        if (e < 8) acc |= fdr->start[e];
        count += (u64a)__builtin_popcount((u32)(~acc & 0xff));
    }
    return count;
}

/* ---- multi-threaded harness (bench.py parity check + cpu_baseline) ---- *
 * The scalar block scan (fdrExec, or noodExec for a noodle table) of one
 * buffer over nthreads contiguous stripes: thread t owns the ends [lo, hi)
 * and scans the window [lo - 7, hi) as its own block from 0, dropping the
 * ends below lo.  Literals are at most 8 bytes (hwlm.h:75) and the FDR start
 * state only touches the first 7 ends of a block (fdr_compile.cpp:129-151),
 * so every owned end sees exactly the single-call result (NOREPEAT aside,
 * which is sequential host state: the digests cover the confirmed set).
 * Output: the match count and the (sum, xor) digest of the (end, id) set. */
#include <pthread.h>
#include <sched.h>

typedef struct {
    const void *eng;
    int nood, simd;
    const u8 *buf;
    size_t len;
    cbctx cb;
    int status;
    int t; /* thread index (pinning) */
} orc_mt_job;

/* optional pinning of the harness threads (bench.py's cpu_baseline: one
 * thread per physical core): thread t runs on g_pin[t % g_npin] */
static int g_pin[1024], g_npin = 0;
void orc_set_pin(const int *cpus, int n) {
    g_npin = n < 0 ? 0 : (n > 1024 ? 1024 : n);
    for (int i = 0; i < g_npin; i++) g_pin[i] = cpus[i];
}
static void orc_pin_self(int t) {
    if (!g_npin) return;
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(g_pin[t % g_npin], &set);
    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

static void *orc_mt_run(void *p) {
    orc_mt_job *j = (orc_mt_job *)p;
    orc_pin_self(j->t);
    if (j->nood) j->status = nood_run((const struct o_nood *)j->eng, j->buf, j->len, 0, &j->cb);
    else j->status = fdr_dispatch_s(j->eng, j->buf, j->len, 0, ~0ULL, &j->cb, j->simd);
    return NULL;
}

/* eng: the engine inside an HWLM blob; nood != 0 for a noodle table; simd:
 * the FDR main zone through get_conf_m128 (bench.py's cpu_baseline) */
long orc_digest_mt2(const void *eng, int nood, int simd, const u8 *buf, size_t len,
                    int nthreads, u64a out[2]);

long orc_digest_mt(const void *eng, int nood, const u8 *buf, size_t len, int nthreads,
                   u64a out[2]) {
    return orc_digest_mt2(eng, nood, 0, buf, len, nthreads, out);
}

long orc_digest_mt2(const void *eng, int nood, int simd, const u8 *buf, size_t len,
                    int nthreads, u64a out[2]) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((size_t)nthreads > len / 64 + 1) nthreads = (int)(len / 64 + 1);
    orc_mt_job jobs[256];
    pthread_t th[256];
    const size_t s = len / (size_t)nthreads;
    for (int t = 0; t < nthreads; t++) {
        const size_t lo = (size_t)t * s, hi = t == nthreads - 1 ? len : lo + s;
        const size_t blo = lo >= 7 ? lo - 7 : 0;
        cbctx cb = {NULL, 0, 0, -1, ~0ULL, 1, lo - blo, blo, 0, 0};
        jobs[t] = (orc_mt_job){eng, nood, simd, buf + blo, hi - blo, cb, 0, t};
        if (pthread_create(&th[t], NULL, orc_mt_run, &jobs[t]) != 0) return -1;
    }
    long n = 0;
    out[0] = out[1] = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].status != 0) n = -1;
        if (n >= 0) n += (long)jobs[t].cb.n;
        out[0] += jobs[t].cb.dsum;
        out[1] ^= jobs[t].cb.dxor;
    }
    return n;
}

/* The same striped scan, keeping every record: (end, id) in the reference's
 * callback order (fdr.c:299-333 per stripe; stripes are contiguous ranges of
 * ends, so their concatenation in stripe order is the single call's order).
 * Writes min(total, cap) records to ends / ids and returns the total (-1 on
 * a failed stripe or allocation).  bench.py's order-exact parity check. */
long orc_records_mt(const void *eng, int nood, const u8 *buf, size_t len, int nthreads,
                    u64a *ends, u32 *ids, size_t cap) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((size_t)nthreads > len / 64 + 1) nthreads = (int)(len / 64 + 1);
    orc_mt_job jobs[256];
    pthread_t th[256];
    const size_t s = len / (size_t)nthreads;
    for (int t = 0; t < nthreads; t++) {
        const size_t lo = (size_t)t * s, hi = t == nthreads - 1 ? len : lo + s;
        const size_t blo = lo >= 7 ? lo - 7 : 0;
        cbctx cb = {NULL, 0, 0, -1, ~0ULL, 2, lo - blo, blo, 0, 0};
        jobs[t] = (orc_mt_job){eng, nood, 0, buf + blo, hi - blo, cb, 0, t};
        if (pthread_create(&th[t], NULL, orc_mt_run, &jobs[t]) != 0) return -1;
    }
    long n = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].status != 0) n = -1;
        for (size_t i = 0; n >= 0 && i < jobs[t].cb.n; i++) {
            if ((size_t)n < cap) {
                ends[n] = jobs[t].cb.out[i].end;
                ids[n] = jobs[t].cb.out[i].id;
            }
            n++;
        }
        free(jobs[t].cb.out);
    }
    return n;
}

/* Many equal blocks (hsbench's corpus of fixed-size chunks): block b =
 * buf[b * blen, min(len, (b + 1) * blen)) scanned as its own hwlmExec call
 * (start 0, no history), every record kept with its block index; blocks are
 * dealt to `nthreads` threads in contiguous ranges and the records come out
 * in block order, each block's in callback order (fdr.c:299-333).  Writes
 * min(total, cap) records (end relative to the block) and returns the total
 * (-1 on a failed block or allocation).  bench.py's cfg-5 proxy parity. */
typedef struct {
    const void *eng;
    int nood;
    const u8 *buf;
    size_t len, blen, b0, b1;
    orc_match *out;
    u32 *blk;
    size_t n, cap;
    int status, t;
} orc_blocks_job;

static void *orc_blocks_run(void *p) {
    orc_blocks_job *j = (orc_blocks_job *)p;
    orc_pin_self(j->t);
    for (size_t b = j->b0; b < j->b1 && j->status == 0; b++) {
        const size_t lo = b * j->blen, hi = lo + j->blen < j->len ? lo + j->blen : j->len;
        cbctx cb = {NULL, 0, 0, -1, ~0ULL, 2, 0, 0, 0, 0};
        j->status = j->nood ? nood_run((const struct o_nood *)j->eng, j->buf + lo, hi - lo, 0, &cb)
                            : fdr_dispatch_s(j->eng, j->buf + lo, hi - lo, 0, ~0ULL, &cb, 0);
        if (j->n + cb.n > j->cap) {
            const size_t nc = 2 * (j->n + cb.n) + 4096;
            orc_match *o = (orc_match *)realloc(j->out, nc * sizeof(orc_match));
            u32 *bk = (u32 *)realloc(j->blk, nc * sizeof(u32));
            if (o) j->out = o;
            if (bk) j->blk = bk;
            if (!o || !bk) j->status = -1;
            else j->cap = nc;
        }
        for (size_t i = 0; j->status == 0 && i < cb.n; i++) {
            j->out[j->n] = cb.out[i];
            j->blk[j->n++] = (u32)b;
        }
        free(cb.out);
    }
    return NULL;
}

long orc_records_blocks(const void *eng, int nood, const u8 *buf, size_t len, size_t blen,
                        int nthreads, u64a *ends, u32 *ids, u32 *blks, size_t cap) {
    if (!blen) return -1;
    const size_t nb = (len + blen - 1) / blen;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((size_t)nthreads > nb) nthreads = nb ? (int)nb : 1;
    orc_blocks_job jobs[256];
    pthread_t th[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (orc_blocks_job){eng, nood, buf, len, blen, nb * (size_t)t / (size_t)nthreads,
                                   nb * (size_t)(t + 1) / (size_t)nthreads, NULL, NULL, 0, 0, 0, t};
        if (pthread_create(&th[t], NULL, orc_blocks_run, &jobs[t]) != 0) return -1;
    }
    long n = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].status != 0) n = -1;
        for (size_t i = 0; n >= 0 && i < jobs[t].n; i++) {
            if ((size_t)n < cap) {
                ends[n] = jobs[t].out[i].end;
                ids[n] = jobs[t].out[i].id;
                blks[n] = jobs[t].blk[i];
            }
            n++;
        }
        free(jobs[t].out);
        free(jobs[t].blk);
    }
    return n;
}

long orc_fdr_count_mt(const void *eng, const u8 *buf, size_t len, int nthreads) {
    u64a d[2];
    return orc_digest_mt(eng, 0, buf, len, nthreads, d);
}
