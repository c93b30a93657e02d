/*
 * flood.cpp — host emulation of the FDR / Teddy flood shortcut
 * (src/fdr/flood_runtime.h:41-335) for the drop-in replay.
 *
 * The reference main loops call floodDetect whenever their pointer passes
 * `tryFloodDetect`.  On a run of one byte c it reports the flood-table ids
 * of c (literals made only of c) at every end of the run, in its own order
 * and without confirm / NOREPEAT, and skips the main loop over those ends;
 * it never changes the matches outside the skipped ends (the stale
 * first-stage state it leaves behind covers only bytes of the same run: the
 * run reaches back at least `suffix` >= the look-back before the check, see
 * flood_compile.cpp:97-104 default suffixes).  Which positions are checked
 * and how far a flood skips depend only on the bytes, the buffer's address
 * (8-byte aligned probes), the engine's loop shape and the flood table —
 * never on the callback — so the events are computed here up front and
 * merged into the replay of the GPU's exact confirm records.
 *
 * Loop shapes (the pointer at each CHECK_FLOOD and the iteration size that
 * bounds a flood):
 *   FDR            fdr.c:663-696 main zone [start + 16, main_end), 16 / 16
 *   Teddy SSE      teddy.c:1004-1066    ptr 16-aligned, +16; step 32
 *   Teddy AVX2     teddy.c:823-888      ptr 32-aligned, +32; step 64
 *   Teddy VBMI     teddy.c:335-388      +64-n_sh; step 64-n_sh, iter 64
 *   Fat AVX2       teddy_avx2.c:593-660 ptr 16-aligned, +16; step 32
 *   Fat VBMI       teddy_avx2.c:395-447 +32-n_sh; step 32-n_sh, iter 32
 * The Teddy build emulated follows vsa_set_accel_vector_size: 16 -> SSE
 * (Fat Teddy needs AVX2: AVX2 shape), 32 -> AVX2, 64 -> AVX-512 VBMI.
 */
#include <cstring>

#include "vsa_internal.h"

namespace vsa {

namespace {

inline u64a load_rounded(const u8 *p) {
    const u8 *q = (const u8 *)(((uintptr_t)p + 7) & ~(uintptr_t)7); /* ROUNDUP_PTR(p, 8) */
    u64a v;
    memcpy(&v, q, 8);
    return v;
}

inline u64a load8(const u8 *p) {
    u64a v;
    memcpy(&v, p, 8);
    return v;
}

/* nextFloodDetect flood_runtime.h:41-83 (64-bit): offset of the first
 * check threshold */
size_t next_flood_detect(const u8 *buf, size_t len) {
    const size_t backoff = 32; /* FLOOD_BACKOFF_START */
    if (len < 256) return len; /* FLOOD_MINIMUM_SIZE */
    if (load_rounded(buf) == load_rounded(buf + 8)) return backoff;
    if (load_rounded(buf + len / 2) == load_rounded(buf + len / 2 + 8)) return backoff;
    if (load_rounded(buf + len - 24) == load_rounded(buf + len - 16)) return backoff;
    return len;
}

/* floodDetect flood_runtime.h:85-335 at the loop pointer i: appends the
 * event (if the run is long enough to skip an iteration) and returns the
 * next threshold; u32 arithmetic as the reference's locals. */
size_t flood_detect(const u8 *buf, size_t len, u32 i, const u8 *fBase, u32 iterBytes,
                    u32 *backoff, std::vector<FloodEvent> &out) {
    const size_t mainLoopLen = len > 2 * (size_t)iterBytes ? len - 2 * (size_t)iterBytes : 0;
    u32 j = i;
    const u8 c = buf[i];
    const u32 fIdx = ((const u32 *)fBase)[c];
    const FDRFlood *fl = (const FDRFlood *)(fBase + sizeof(u32) * 256) + fIdx;
    const u64a cmpVal = 0x0101010101010101ULL * c;
    const u64a probe = load_rounded(buf + i);
    if (probe != cmpVal || fl->idCount >= FDR_FLOOD_MAX_IDS) {
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
        if (load8(buf + j) != cmpVal || load8(buf + j + 8) != cmpVal ||
            load8(buf + j + 16) != cmpVal || load8(buf + j + 24) != cmpVal)
            break;
    }
    for (; j + 8 < mainLoopLen; j += 8) {
        if (load8(buf + j) != cmpVal) break;
    }
    for (; j < mainLoopLen; j++) {
        if (buf[j] != c) break;
    }
    if (j > i) {
        j--;
        const u32 floodSize = ((j - i) / iterBytes) * iterBytes;
        if (floodSize) out.push_back(FloodEvent{i, floodSize, fl});
    } else {
        *backoff *= 2;
    }
floodout:
    if ((size_t)(u32)(j + *backoff) < mainLoopLen - 128) {
        return (size_t)(i > j ? i : j) + *backoff;
    }
    return mainLoopLen;
}

struct Shape {
    size_t p;    /* pointer (offset) at the first CHECK_FLOOD */
    size_t step; /* loop increment */
    size_t body; /* loop runs while p + body <= end */
    size_t end;
    u32 iter;    /* iterBytes handed to floodDetect */
};

size_t roundup(const u8 *buf, size_t off, size_t n) {
    const uintptr_t a = (uintptr_t)buf + off;
    return off + (size_t)(((a + n - 1) & ~(uintptr_t)(n - 1)) - a);
}

/* Teddy loop shapes: prologue blocks, then the main loop */
bool teddy_shape(const u8 *buf, size_t len, size_t start, u32 engineID, u32 vsize, Shape *s) {
    const bool fat = engineID >= 3 && engineID <= 10;
    const u32 nmasks = fat ? (engineID - 3) / 2 + 1 : (engineID - 11) / 2 + 1;
    size_t p = start;
    if (vsize >= 64) {
        /* VBMI: one head block of loopBytes, then overlapping loads */
        const size_t L = (fat ? 32 : 64) - (nmasks - 1);
        if (p + L <= len) p += L;
        *s = Shape{p, L, L, len, fat ? 32u : 64u};
        return true;
    }
    const size_t blk = (!fat && vsize == 32) ? 32 : 16; /* AVX2 Teddy works in 32-B halves */
    const size_t ms = roundup(buf, p, blk);
    if (p < ms) p = ms;
    if (p + blk <= len) p += blk;
    *s = Shape{p, 2 * blk, 2 * blk, len, (u32)(2 * blk)};
    return true;
}

} // namespace

void flood_events(const u8 *buf, size_t len, size_t start, const u8 *eng, u32 vsize,
                  std::vector<FloodEvent> &out) {
    out.clear();
    if (start >= len) return;
    const u32 engineID = ((const u32 *)eng)[0];
    const u32 floodOffset = ((const u32 *)eng)[5];
    const u8 *fBase = eng + floodOffset;
    size_t tfd = next_flood_detect(buf, len);
    if (tfd >= len) return; /* never reached by a loop pointer */
    Shape s;
    if (engineID == 0) {
        /* prepareZones fdr.c:625-659: only the main zone checks floods
         * (start / end / short zones point floodPtr past their buffer) */
        if (len - start <= 16) return;
        const size_t p0 = start + 16;
        const size_t main_end = start + ((len - start - 3) / 16) * 16;
        if (main_end <= p0) return;
        s = Shape{p0, 16, 16, main_end, 16};
    } else if ((engineID >= 3 && engineID <= 10) || (engineID >= 11 && engineID <= 18)) {
        teddy_shape(buf, len, start, engineID, vsize, &s);
    } else {
        return;
    }
    u32 backoff = 32;
    size_t p = s.p;
    while (p + s.body <= s.end) {
        if (p <= tfd) {
            /* next loop pointer strictly past the threshold */
            p += ((tfd - p) / s.step + 1) * s.step;
            continue;
        }
        const size_t before = out.size();
        tfd = flood_detect(buf, len, (u32)p, fBase, s.iter, &backoff, out);
        if (out.size() != before) p += out.back().size; /* ptr += floodSize */
        p += s.step;
    }
}

} // namespace vsa
