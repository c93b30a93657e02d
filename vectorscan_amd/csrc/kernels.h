/*
 * kernels.h — host/device shared parameter blocks for the MI355X kernels.
 * Plain structs only (passed by value as kernel arguments).
 */
#ifndef VSA_KERNELS_H
#define VSA_KERNELS_H

#include <stdint.h>

/* One hwlmExec-equivalent block inside a device batch.  All offsets are
 * relative to the batch's data pointer. */
struct VsaBlock {
    uint64_t base;      /* first byte of the block (its buf[0]) */
    uint64_t len;       /* block length */
    uint64_t start;     /* hwlmExec `start` (ends < start are not reported) */
    uint64_t seg_first; /* index of the block's first segment */
    int64_t zbase;      /* FDR: first looked-up position (start, or len - 16
                           for a short zone; may be < 0).  The start state
                           always applies from `start`. */
    int64_t org;        /* aligned (1 KiB, relative to data & ~15) origin of
                           the block's first segment */
    int64_t rlo;        /* ends < rlo are not reported either; unlike `start`
                           it does not move the FDR start state (a stripe
                           window [lo - 7, hi) keeps ends >= 7 of a block
                           scanned from its own first byte, stripe.py) */
    uint64_t hlen;      /* streaming: len_history (confirm overhang bound,
                           fdr_confirm_runtime.h:79-88); 0 = block mode */
    uint32_t hist;      /* bytes readable before base (min(hlen, 16)) */
    uint32_t flags;     /* VSA_BLK_* */
};
#ifdef __cplusplus
static_assert(sizeof(VsaBlock) == 72, "VsaBlock layout (vsa_plan_blocks, tests/test_plan.py)");
#endif

/* The block is a streaming call with history (fdrExecStreaming fdr.c:827,
 * len_history > 0): no FDR start state, the look-back starts one byte
 * before `start` (getInitState fdr.c:129-142), Teddy / noodle read up to
 * nMasks - 1 / msk_len - 1 history bytes. */
#define VSA_BLK_STREAM 1u
/* Set on the first block of a packed segment whose blocks (2-128 of them)
 * are back to back in memory, scanned from their first byte (start 0, no
 * report_lo) and >= 1 KiB each: FDR / Teddy scan the segment as one range
 * and the confirm places each end in its block (kernels.hip "runs").  A
 * streaming block in a run reads its history from the bytes before it,
 * which are its predecessor's in the layouts that make runs. */
#define VSA_BLK_RUN 2u
#define VSA_RUN_MAX 128u
#define VSA_RUN_MIN_LEN 1024u

/* A confirmed literal match.  `key` sorts into the reference callback order:
 * end (bits 63..24), bucket (23..20), LitInfo offset within its bucket's
 * confirm structure in 8-byte units (19..0; LitInfo is 8-aligned,
 * fdr_confirm_compile.cpp:256) — fdr.c:299-333 / teddy_runtime_common.h:419-440
 * walk candidates LSB-first (end, then bucket) and each chain in memory
 * order. */
#define VSA_KEY_END_SHIFT 24
#define VSA_KEY_BUCKET_SHIFT 20
#define VSA_KEY_LI_MASK 0xfffffu

/* Key of the 4-field derived FDR first stage (VSA_MODE_FDR4, runtime.hip
 * derive_fdr4_table) at position p, from the bytes b2 = b[p-2], b1 =
 * b[p-1], b0 = b[p]: 15 bits, the low 7 bits of b1, bit 0 of b2, then the
 * low 7 bits of b0 -- the 16-bit pair (b1, b0) as it lies in memory with its
 * two bit-7s replaced (kernels.hip fdr4_keys builds two per dword in three
 * ops). */
#ifdef __HIPCC__
__host__ __device__
#endif
static inline uint32_t vsa_fdr4_key(uint32_t b2, uint32_t b1, uint32_t b0) {
    return (b1 & 0x7fu) | ((b2 & 1u) << 7) | ((b0 & 0x7fu) << 8);
}

enum VsaLitMode {
    VSA_MODE_TEDDY = 1, /* 4 lanes x 8 buckets, 1-byte key */
    VSA_MODE_FAT = 2,   /* 4 lanes x 16 buckets, 1-byte key */
    VSA_MODE_NOOD = 3,  /* noodle: masked compare of the <= 8 bytes ending at e */
    VSA_MODE_FDR4 = 4,  /* FDR engines, 4 fields x 8 buckets (u32), 3-byte key */
};

/* binned sort of the match records: bins by the end's top bits, each bin
 * sorted by one wave when no bin holds more than VSA_SORT_BIN_MAX */
#define VSA_SORT_BIN_BITS 14
#define VSA_SORT_BINS (1u << VSA_SORT_BIN_BITS)
#define VSA_LBINS 256u /* sort bins a workgroup may count in LDS */
#define VSA_SORT_BIN_MAX 64
#define VSA_CTR_BIN_OVERFLOW 12 /* counters[12]: some bin passed VSA_SORT_BIN_MAX */
#define VSA_FIN_MAX_GRID 1024u /* workgroups of a fused-finish launch, at most */

struct VsaLitParams {
    const uint8_t *data;
    const VsaBlock *blocks;
    uint32_t nblocks;
    uint64_t nsegs;
    const uint32_t *seg_desc; /* 4 words per segment: first block | count <<
                                 24, offset and length in KiB from the block
                                 origin (a part of one block), 0 */
    const uint32_t *wg_seg;   /* workgroup b's segments are [wg_seg[b],
                                 wg_seg[b + 1]), handed out in LDS */
    const uint32_t *wg_bins;  /* [2b, 2b + 1]: the sort bins workgroup b owns
                                 alone (runtime.hip plan_wg_bins), counted in
                                 LDS; others with global atomics */
    uint32_t steal;           /* a wave out of segments steals sweep groups
                                 inside its workgroup when some wave has at
                                 least `steal` unclaimed (0: off) */
    const uint64_t *table;  /* FDR4 table (u32 entries) / Teddy byte table */
    uint32_t table_entries;
    uint32_t dmask;
    uint32_t end_par;       /* FDR4 split passes: 0 every end; 1 / 2 only the
                               ends whose byte has bit 0 clear / set */
    uint64_t state_lo, state_hi; /* FDR start state (fdr->start) */
    const uint8_t *conf_base;    /* engine confBase (device) */
    uint32_t conf_off[16];       /* confBase[b], 0 = empty bucket */
    const uint32_t *slotmap;     /* per-bucket bitmap of litIndex[h] != 0 */
    uint32_t slot_words;
    uint32_t slot_off[16];       /* word offset per bucket, ~0 = no prefilter */
    uint8_t slot_bits[16];       /* bits of the prefilter hash per bucket (the
                                    bucket's nBits, fewer when coarsened) */
    uint64_t nood_msk, nood_cmp; /* noodle msk / cmp << 8 * (8 - msk_len) */
    uint32_t nood_len, nood_id;  /* noodTable msk_len, id */
    uint64_t pf_mult;            /* FDRConfirm.mult shared by the prefiltered
                                    buckets (fdr_confirm_compile.cpp) */
    uint32_t qcap;               /* per-wave LDS confirm-queue entries */
    uint32_t nconf;              /* confirm waves per workgroup (1..4); the
                                    other LIT_WAVES - nconf waves scan */
    uint32_t dbg;                /* debug: bit0 verify queued keys against HBM
                                    (mismatches -> counters[3]); bit1 drop all
                                    candidates (filter-only timing); bit3 stop
                                    after the candidate test; bit4 skip the
                                    push; bit5 count first-stage candidates;
                                    bit6 confirm-wave phase counters; bit7
                                    the confirm wave drops what it gathers;
                                    bit8 32-B ring entries (drops the data);
                                    bit10 confirm wave at base priority */
    uint64_t *out_keys;
    uint32_t *out_ids;
    uint64_t out_cap;
    uint32_t *bin_counts;        /* binned sort: records per bin of end >>
                                    bin_shift, counted as they are emitted
                                    (nullptr: no binned sort) */
    uint32_t bin_shift;
    uint64_t *bin_keys;          /* staged binned sort (vsa_bin_finish):
                                    record s of bin b (its key here, its id
                                    in bin_ids) goes to [b * VSA_SORT_BIN_MAX
                                    + s] (s from the bin's count; a bin past
                                    VSA_SORT_BIN_MAX sets
                                    counters[VSA_CTR_BIN_OVERFLOW]).  The
                                    records then live only there: out_keys /
                                    out_ids are not written and counters[0]
                                    is only counted (no output slot) */
    uint32_t *bin_ids;
    unsigned long long *wg_time;  /* schedule feedback (or null): [b] = xcc <<
                                     60 | end of workgroup b's scanning
                                     waves, [grid + b] = its entry (100 MHz) */
    unsigned long long *wave_log; /* diagnostic (dbg bit12): 8 u64 per scanning
                                     wave: start, end (100 MHz), segments,
                                     KiB iterations, workgroup, wave, XCC, HW_ID */
    unsigned long long *counters; /* [0] matches, [2] candidates handed to
                                     confirm (after the slot prefilter;
                                     diagnostic) */
    /* Fused finish (kernels.hip fused_finish; fin_keys null = off): each
     * workgroup bins its records over its own end range in LDS-counted local
     * bins (staging row blockIdx.x * VSA_LBINS + bin of bin_keys / bin_ids),
     * sorts them at its end and writes them at its offset, found by a
     * look-back over the lower workgroups' totals; the last workgroup out
     * publishes the counters.  No vsa_bin_finish launch. */
    const uint32_t *fin_wg;       /* 4 words per workgroup: lowest end (lo,
                                     hi word), local bin shift, local bins */
    uint64_t *fin_keys;           /* the sorted records (out_cap) */
    uint32_t *fin_ids;
    unsigned long long *fin_agg;  /* [2b] = epoch << 32 | crowded << 31 |
                                     workgroup b's records, [2b + 1] = epoch
                                     << 32 | its confirm candidates */
    uint32_t fin_epoch;           /* this launch's tag in fin_agg (nonzero) */
    unsigned long long *fin_pub;  /* host publish block (vsa_publish layout) */
    unsigned long long fin_seq;
    uint64_t *fin_pk;             /* packed collective buffer (or null) */
    uint64_t fin_pk_cap;
    /* Dynamic shares (kernels.hip dyn_bounds; dyn_kib 0 = off): workgroup
     * b scans the KiB range [L_b, L_b+1) of the plan's live KiB (descriptor
     * word 3 = a segment's KiB position), L from per-XCD weights it derives
     * at its start from the previous launch's end times, each L held within
     * dyn_margin KiB of the equal-share boundary floor(dyn_kib * b / grid) */
    const unsigned long long *dyn_prev; /* the previous such launch's records
                                           (wg_time's layout) or null: equal */
    const uint32_t *dyn_wprev;          /* ... its weights (8, 16.16) */
    uint32_t *dyn_wout;                 /* this launch's (workgroup 0 writes) */
    uint32_t dyn_kib;
    uint32_t dyn_margin;
};


/* Byte-class scan (shufti / truffle / vermicelli reduce to a 256-bit class).
 * pair != 0: position i is set when cls[b[i]] && cls2[b[i+1]] (double
 * vermicelli / double shufti without the partial-at-end rule, applied on the
 * host). */
struct VsaClassParams {
    const uint8_t *data;
    uint64_t len;
    uint32_t cls[8];
    uint32_t cls2[8];
    int pair;
    uint64_t *bitmap;              /* (len + 63) / 64 words, may be null */
    unsigned long long *first;     /* [slots] atomicMin of first set index */
    unsigned long long *last;      /* [slots] atomicMax of (last set index + 1) */
    unsigned long long *count;     /* [slots] popcount of the bitmap */
    uint32_t slots;                /* workgroup b updates slot b % slots, at
                                      u64 index 16 * slot (one line each) */
};

/* Double shufti (shuftiDoubleExec): bucketed byte-pair test with the
 * reference's per-block lane artifacts (see orc_shufti_double / kernel).
 * first[0..2] receive atomicMin of the first match of the head, aligned and
 * tail stages (initialised to ~0). */
struct VsaPairParams {
    const uint8_t *data;
    uint64_t len;
    uint8_t n1[256], n2[256]; /* bucket sets: ~(lo[c & 15] | hi[c >> 4]) */
    uint32_t vsize;           /* VECTORSIZE S (16, 32, 64) */
    uint32_t mis;             /* buffer address mod S */
    unsigned long long *first; /* [3], one 128-B line apart (stride 16) */
};

#endif
