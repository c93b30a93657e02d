/*
 * dropin.hip -- the host half of the drop-in boundary (SURVEY.md section 8
 * rows a1-a14, b): the reference's own entry points with their signatures
 * (hwlmExec hwlm.h:116, fdrExec fdr.h:58, noodExec noodle_engine.h:47, the
 * streaming forms, shuftiExec shufti.h:46-55, truffleExec truffle.h:45-49,
 * the vermicelli family vermicelli.hpp:47-95, run_accel accel.h:148), the
 * per-thread blob registry, the replay of the GPU's confirmed records
 * through the callback with confWithBit's sequential state
 * (fdr_confirm_runtime.h:43-102: NOREPEAT, groups / control, termination,
 * the INCLUDED_JUMP squash of program_runtime.c:2985-2997, the flood
 * shortcut's reports), the accel pre-skip (hwlm.c:48-105), the bridge
 * hs_lit.cpp runs on (namespace vsa) and the builder API.
 */
#include "runtime_internal.h"

namespace vsa_rt {

uint32_t g_vector_size = 64;

/* ------------------------------------------------------------ registry */

thread_local vsa_ctx *t_ctx = nullptr;

vsa_ctx *default_ctx() {
    if (!t_ctx) {
        int dev = 0;
        const char *e = getenv("VSA_DEVICE");
        if (e) dev = atoi(e);
        if (vsa_ctx_create(dev, &t_ctx) != VSA_OK) t_ctx = nullptr;
    }
    return t_ctx;
}

/* Keyed by (pointer, size); a lookup of an unregistered blob also compares
 * the whole blob with the cached host copy, so a database freed and
 * re-allocated at the same address is never served from a stale device
 * copy (memcmp runs at memory speed, ~20 us for a 0.4 MB FDR blob).  A blob
 * registered with vsa_hwlm_register is immutable until its unregister (the
 * integration registers it where the database is loaded),
 * so its lookups skip the compare. */
std::mutex g_reg_mu;
std::map<const void *, size_t> g_registered; /* pointer -> size */

bool is_registered(const void *p, size_t size) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_registered.find(p);
    return it != g_registered.end() && it->second == size;
}

thread_local std::map<RegKey, vsa_db *> t_registry;

size_t engine_size(const uint8_t *eng, int type) {
    if (type == HWLM_ENGINE_NOOD) return sizeof(noodTable);
    return ((const uint32_t *)eng)[1]; /* FDR.size / Teddy.size */
}

/* look up (or upload) the device copy of a blob given as HWLM or as a bare
 * engine (type = -1: HWLM header present) */
vsa_db *registry_get(const void *ptr, int bare_type) {
    vsa_ctx *c = default_ctx();
    if (!c) return nullptr;
    const uint8_t *p = (const uint8_t *)ptr;
    size_t size;
    int type;
    if (bare_type < 0) {
        type = p[0];
        size = VSA_ROUNDUP_CL(sizeof(HWLM)) + engine_size(p + VSA_ROUNDUP_CL(sizeof(HWLM)), type);
    } else {
        type = bare_type;
        size = engine_size(p, type);
    }
    RegKey k{ptr, size};
    auto it = t_registry.find(k);
    if (it != t_registry.end()) {
        vsa_db *old = it->second;
        const uint8_t *cached = old->hblob + (bare_type < 0 ? 0 : VSA_ROUNDUP_CL(sizeof(HWLM)));
        if (is_registered(ptr, size) || memcmp(cached, p, size) == 0) return old;
        vsa_db_free(old); /* erases the registry entry */
    }
    vsa_db *db = nullptr;
    int r;
    if (bare_type < 0) {
        r = vsa_db_load(c, ptr, size, &db);
    } else {
        /* wrap the bare engine in an HWLM header */
        size_t tot = VSA_ROUNDUP_CL(sizeof(HWLM)) + size;
        std::vector<uint8_t> tmp(tot + 64, 0);
        uint8_t *al = (uint8_t *)VSA_ROUNDUP_N((uintptr_t)tmp.data(), 64);
        al[0] = (uint8_t)type;
        memcpy(al + VSA_ROUNDUP_CL(sizeof(HWLM)), p, size);
        r = vsa_db_load(c, al, tot, &db);
    }
    if (r != VSA_OK) return nullptr;
    t_registry[k] = db;
    return db;
}

/* ----------------------------------------------------------- replay --- */

/* offsets inside struct hs_scratch (src/scratch.h:172-219), x86-64 */
struct ScratchLayoutProbe {
    struct RoseContext_ {
        uint8_t mpv_inactive;
        uint64_t groups, lit_offset_adjust, delayLastEndOffset, lastEndOffset,
            lastMatchOffset, lastCombMatchOffset, minMatchOffset,
            minNonMpvMatchOffset, next_mpv_offset;
        uint32_t filledDelayedSlots, curr_qi;
        const uint8_t *ll_buf;
        size_t ll_len;
        const uint8_t *ll_buf_nocase;
        size_t ll_len_nocase;
    };
    struct catchup_pq_ {
        void *qm;
        uint32_t qm_size;
    };
    struct core_info_ {
        void *userContext;
        void *userCallback;
        const void *rose;
        char *state, *exhaustionVector, *logicalVector, *combVector;
        const uint8_t *buf;
        size_t len;
        const uint8_t *hbuf;
        size_t hlen;
        uint64_t buf_offset;
        uint8_t status;
    };
    struct match_deduper_ {
        void *log[2];
        void *som_log[2];
        uint64_t *som_start_log[2];
        uint32_t dkey_count, log_size;
        uint64_t current_report_offset;
        uint8_t som_log_dirty;
    };
    uint32_t magic;
    uint8_t in_use;
    uint32_t queueCount, activeQueueArraySize, bStateSize, tStateSize, fullStateSize;
    RoseContext_ tctxt;
    char *bstate, *tstate, *fullState;
    void *queues, *aqa, **delay_slots, **al_log;
    uint64_t al_log_sum;
    catchup_pq_ catchup_pq;
    core_info_ core_info;
    match_deduper_ deduper;
    uint32_t anchored_literal_region_len, anchored_literal_fatbit_size;
    void *handled_roles;
    uint64_t *som_store, *som_attempted_store;
    void *som_set_now, *som_attempted_set;
    uint64_t som_set_now_offset;
    uint32_t som_store_count, som_fatbit_size, handledKeyFatbitSize, delay_fatbit_size,
        scratchSize;
    char *scratch_alloc;
    uint64_t *fdr_conf;
    uint8_t fdr_conf_offset;
};

std::atomic<long> g_core_buf_off{(long)(offsetof(ScratchLayoutProbe, core_info) +
                                        offsetof(ScratchLayoutProbe::core_info_, buf))};
std::atomic<long> g_core_hbuf_off{(long)(offsetof(ScratchLayoutProbe, core_info) +
                                         offsetof(ScratchLayoutProbe::core_info_, hbuf))};
std::atomic<long> g_core_hlen_off{(long)(offsetof(ScratchLayoutProbe, core_info) +
                                         offsetof(ScratchLayoutProbe::core_info_, hlen))};
std::atomic<long> g_fdr_conf_off{(long)offsetof(ScratchLayoutProbe, fdr_conf)};
std::atomic<long> g_fdr_conf_offset_off{(long)offsetof(ScratchLayoutProbe, fdr_conf_offset)};

hwlm_error_t replay_nood(const uint64_t *keys, const uint32_t *ids, uint64_t n,
                         HWLMCallback cb, hs_scratch *scratch) {
    for (uint64_t i = 0; i < n; i++) {
        if (cb(keys[i] >> VSA_KEY_END_SHIFT, ids[i], scratch) == HWLM_TERMINATE_MATCHING) {
            return HWLM_TERMINATED;
        }
    }
    return HWLM_SUCCESS;
}

/* the flood shortcut's reports (flood_runtime.h:191-319): per group of
 * S = 4 (idCount <= 2) or 2 ends, each end reports every flood id whose
 * groups meet the live control, the run stopping once control leaves
 * allGroups; no confirm, no NOREPEAT */
bool emit_flood(const vsa::FloodEvent &ev, HWLMCallback cb, hs_scratch *scratch,
                uint64_t &control) {
    const FDRFlood *fl = ev.fl;
    if (fl->idCount && (control & fl->allGroups)) {
        const uint32_t S = fl->idCount <= 2 ? 4 : 2;
        for (uint32_t t = 0; t < ev.size && (control & fl->allGroups); t += S)
            for (uint32_t k = 0; k < S; k++)
                for (uint32_t d = 0; d < fl->idCount; d++)
                    if (control & fl->groups[d])
                        control = cb((size_t)(ev.i + t + k), fl->ids[d], scratch);
    }
    return control != HWLM_TERMINATE_MATCHING;
}

/* The confirmed records of one call, in reference order, through the
 * callback with confWithBit's sequential state; `floods` (ascending) replace
 * the ends they skip. */
hwlm_error_t replay_lit(const vsa_db *db, const uint64_t *keys, uint64_t n,
                        HWLMCallback cb, hs_scratch *scratch, hwlm_group_t groups,
                        const std::vector<vsa::FloodEvent> *floods,
                        bool scratch_is_real) {
    const uint8_t *eng = db->hblob + VSA_ROUNDUP_CL(sizeof(HWLM));
    const uint8_t *confBase = eng + ((const uint32_t *)eng)[4];
    const bool squash_ok = scratch && scratch_is_real && db->mode == VSA_MODE_FDR4;
    const long co = g_fdr_conf_off.load(), coo = g_fdr_conf_offset_off.load();
    const size_t nf = floods ? floods->size() : 0;
    size_t fe = 0;
    uint64_t skip_lo = 0, skip_hi = 0; /* ends a flood replaced */
    uint64_t control = groups;
    uint32_t last_match = ~0u;
    uint64_t i = 0;
    while (i < n || fe < nf) {
        const uint64_t end = i < n ? keys[i] >> VSA_KEY_END_SHIFT : ~0ULL;
        if (fe < nf && (*floods)[fe].i <= end) {
            const vsa::FloodEvent &ev = (*floods)[fe++];
            if (!emit_flood(ev, cb, scratch, control)) return HWLM_TERMINATED;
            skip_lo = ev.i;
            skip_hi = (uint64_t)ev.i + ev.size;
            continue;
        }
        uint64_t j = i;
        while (j < n && (keys[j] >> VSA_KEY_END_SHIFT) == end) j++;
        if (end >= skip_lo && end < skip_hi) {
            i = j;
            continue;
        }
        uint32_t squashed = 0;
        for (uint64_t k = i; k < j; k++) {
            const uint32_t b = (uint32_t)(keys[k] >> VSA_KEY_BUCKET_SHIFT) & 15;
            const uint32_t lidx = (uint32_t)(keys[k] & VSA_KEY_LI_MASK);
            if (squashed & (1u << b)) continue;
            const LitInfo *li =
                (const LitInfo *)(confBase + db->conf_off[b] + (size_t)lidx * 8);
            if (last_match == li->id && (li->flags & FDR_LIT_FLAG_NOREPEAT)) continue;
            if (!(li->groups & control)) continue;
            last_match = li->id;
            if (squash_ok && co >= 0) {
                /* live conf word: later buckets still pending at this end */
                uint64_t conf = 0;
                for (uint64_t m = k + 1; m < j; m++) {
                    uint32_t bb = (uint32_t)(keys[m] >> VSA_KEY_BUCKET_SHIFT) & 15;
                    if (bb > b) conf |= 1ull << bb;
                }
                const uint64_t before = conf;
                uint64_t **slot = (uint64_t **)((char *)scratch + co);
                *slot = &conf;
                *((uint8_t *)scratch + coo) = (uint8_t)b;
                control = cb(end, li->id, scratch);
                *slot = nullptr;
                squashed |= (uint32_t)(before & ~conf);
            } else {
                control = cb(end, li->id, scratch);
            }
            if (control == HWLM_TERMINATE_MATCHING) return HWLM_TERMINATED;
        }
        i = j;
    }
    return HWLM_SUCCESS;
}

/* flood events of one call when the blob's flood table is live */
const std::vector<vsa::FloodEvent> *floods_for(const vsa_db *db, const uint8_t *buf, size_t len,
                                               size_t start,
                                               std::vector<vsa::FloodEvent> &ev) {
    if (!db->flood_live || db->type != HWLM_ENGINE_FDR) return nullptr;
    vsa::flood_events(buf, len, start, db->hblob + VSA_ROUNDUP_CL(sizeof(HWLM)),
                      g_vector_size, ev);
    return ev.empty() ? nullptr : &ev;
}

/* the last drop-in scan's n records on the host, in reference order: from
 * the published copy (vsa_publish, <= PUB_RECS records) or the device */
int fetch_records(vsa_ctx *c, uint64_t n, std::vector<uint64_t> &keys,
                  std::vector<uint32_t> &ids) {
    keys.resize(n);
    ids.resize(n);
    if (!n) return VSA_OK;
    if (c->launch.published && (c->launch.flags & SCAN_HOST_SORT_SMALL) && c->host_sort &&
        n <= PUB_RECS) {
        const unsigned long long *h = c->ws.h_pub;
        memcpy(keys.data(), h + 17, n * 8);
        memcpy(ids.data(), (const uint32_t *)(h + 17 + PUB_RECS), n * 4);
    } else {
        VSA_CHECK(hipMemcpyAsync(keys.data(), c->ws.d_keys[c->cur], n * 8,
                                 hipMemcpyDeviceToHost, c->stream));
        VSA_CHECK(hipMemcpyAsync(ids.data(), c->ws.d_ids[c->cur], n * 4,
                                 hipMemcpyDeviceToHost, c->stream));
        VSA_CHECK(hipStreamSynchronize(c->stream));
    }
    if (c->host_sort && n > 1) {
        /* keys are unique (end, bucket, LitInfo) */
        std::vector<std::pair<uint64_t, uint32_t>> kv(n);
        for (uint64_t i = 0; i < n; i++) kv[i] = {keys[i], ids[i]};
        std::sort(kv.begin(), kv.end());
        for (uint64_t i = 0; i < n; i++) {
            keys[i] = kv[i].first;
            ids[i] = kv[i].second;
        }
    }
    return VSA_OK;
}

/* scan one host buffer with the default context */
/* One hwlmExec-equivalent scan of a host buffer.  hend != NULL: streaming
 * with history (the 16 bytes before hend are copied in front of buf, as
 * the reference reads them, fdr.c:380-560). */
int scan_host(vsa_db *db, const uint8_t *buf, size_t len, size_t start,
              std::vector<uint64_t> &keys, std::vector<uint32_t> &ids,
              const uint8_t *hend, size_t hlen) {
    vsa_ctx *c = db->ctx;
    int r;
    const size_t pre = hend ? 16 : 0;
    const bool resident = !pre && c->res_host == buf && c->res_len == len;
    if (!resident) c->res_host = nullptr;
    if ((r = ensure_in(c, pre + len + 16)) != VSA_OK) return r;
    if (!resident && pre + len <= PIN_STAGE_MAX) {
        /* history + block staged in pinned memory, one DMA */
        if ((r = ensure_hin(c, pre + len)) != VSA_OK) return r;
        if (pre) memcpy(c->ws.h_in, hend - 16, 16);
        if (len) memcpy(c->ws.h_in + pre, buf, len);
        VSA_CHECK(hipMemcpyAsync(c->ws.d_in, c->ws.h_in, pre + len, hipMemcpyHostToDevice,
                                 c->stream));
    } else {
        if (pre) {
            VSA_CHECK(hipMemcpyAsync(c->ws.d_in, hend - 16, 16, hipMemcpyHostToDevice,
                                     c->stream));
        }
        if (len && !resident) {
            VSA_CHECK(hipMemcpyAsync(c->ws.d_in + pre, buf, len, hipMemcpyHostToDevice,
                                     c->stream));
        }
    }
    uint64_t off = 0, l = len, st = start, n = 0, hl = hlen;
    if ((r = scan_blocks_impl(c, db, c->ws.d_in + pre, &off, &l, &st, 1, SCAN_HOST_SORT_SMALL,
                              &n, pre ? &hl : nullptr)) != VSA_OK)
        return r;
    return fetch_records(c, n, keys, ids);
}

/* class scan over a host buffer: returns first / last+1 */
int class_host(const uint8_t cls[32], const uint8_t *cls2, const uint8_t *buf, size_t len,
               uint64_t *first, uint64_t *last) {
    vsa_ctx *c = default_ctx();
    if (!c) return VSA_E_DEVICE;
    uint64_t cnt;
    if (c->res_host && buf >= c->res_host && buf + len <= c->res_host + c->res_len) {
        /* inside the buffer this drop-in call already uploaded (hwlmExec
         * reserved twice its size): scan it in place when 16-B aligned,
         * else from an aligned device-side copy behind it */
        const uint8_t *d = c->ws.d_in + (buf - c->res_host);
        if ((uintptr_t)d & 15) {
            uint8_t *cp = c->ws.d_in + ((c->res_len + 16 + 15) & ~(size_t)15);
            if (cp + len > c->ws.d_in + c->ws.in_cap) return VSA_E_INVALID;
            VSA_CHECK(hipMemcpyAsync(cp, d, len, hipMemcpyDeviceToDevice, c->stream));
            d = cp;
        }
        return vsa_class_scan(c, cls, cls2, d, len, nullptr, first, last, &cnt, 0);
    }
    c->res_host = nullptr;
    int r;
    if ((r = ensure_in(c, len + 16)) != VSA_OK) return r;
    if (len) {
        VSA_CHECK(hipMemcpyAsync(c->ws.d_in, buf, len, hipMemcpyHostToDevice, c->stream));
    }
    return vsa_class_scan(c, cls, cls2, c->ws.d_in, len, nullptr, first, last, &cnt, 0);
}

/* shuftiDoubleExec on the device (VsaPairParams); `vsize` = the reference
 * build's VECTORSIZE, the buffer's host address fixes the block alignment. */
int64_t pair_host(const uint8_t *lo1, const uint8_t *hi1, const uint8_t *lo2,
                  const uint8_t *hi2, const uint8_t *buf, size_t len, uint32_t vsize) {
    vsa_ctx *c = default_ctx();
    if (!c) return -2;
    if (!len) return 0;
    if (ensure_in(c, len + 16) != VSA_OK) return -2;
    Workspace &w = c->ws;
    if (hipMemcpyAsync(w.d_in, buf, len, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return -2;
    unsigned long long *first = w.d_counters + PAIR_BASE;
    if (hipMemsetAsync(first, 0xff, 48 * 8, c->stream) != hipSuccess) return -2;
    VsaPairParams P;
    memset(&P, 0, sizeof(P));
    P.data = w.d_in;
    P.len = len;
    for (int ch = 0; ch < 256; ch++) {
        P.n1[ch] = (uint8_t)~(lo1[ch & 15] | hi1[ch >> 4]);
        P.n2[ch] = (uint8_t)~(lo2[ch & 15] | hi2[ch >> 4]);
    }
    P.vsize = vsize;
    P.mis = (uint32_t)((uintptr_t)buf % vsize);
    P.first = first;
    uint64_t want = (len + 255) / 256;
    uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)c->num_cus * 4));
    drop_stale_error();
    hipLaunchKernelGGL(vsa_pair_scan, dim3(grid), dim3(256), 0, c->stream, P);
    if (hipGetLastError() != hipSuccess) return -2;
    if (hipMemcpyAsync(w.h_counters + PAIR_BASE, first, 48 * 8, hipMemcpyDeviceToHost,
                       c->stream) != hipSuccess)
        return -2;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return -2;
    const unsigned long long *h = w.h_counters + PAIR_BASE;
    if (h[0] != ~0ULL) return (int64_t)h[0];
    if (h[16] != ~0ULL) return (int64_t)h[16];
    if (h[32] != ~0ULL && h[32] < len) return (int64_t)h[32];
    return (int64_t)len;
}

void cls_from_shufti(const uint8_t *lo, const uint8_t *hi, uint8_t cls[32]) {
    memset(cls, 0, 32);
    for (int ch = 0; ch < 256; ch++) {
        if (lo[ch & 15] & hi[ch >> 4]) cls[ch >> 3] |= (uint8_t)(1u << (ch & 7));
    }
}

void cls_from_truffle(const uint8_t *m1, const uint8_t *m2, uint8_t cls[32]) {
    memset(cls, 0, 32);
    for (int ch = 0; ch < 256; ch++) {
        const uint8_t *m = (ch & 0x80) ? m2 : m1;
        if ((m[ch & 15] >> ((ch >> 4) & 7)) & 1) cls[ch >> 3] |= (uint8_t)(1u << (ch & 7));
    }
}

void cls_from_masked(uint8_t c, uint8_t m, bool negate, uint8_t cls[32]) {
    memset(cls, 0, 32);
    for (int ch = 0; ch < 256; ch++) {
        bool in = ((uint8_t)ch & m) == c;
        if (in != negate) cls[ch >> 3] |= (uint8_t)(1u << (ch & 7));
    }
}

bool cls_has(const uint8_t cls[32], uint8_t ch) { return (cls[ch >> 3] >> (ch & 7)) & 1; }

} // namespace vsa_rt

extern "C" {

/* run_hwlm_accel hwlm.c:48-80 (no minimum length, no offset) */
static const uint8_t *hwlm_accel(const union AccelAux *a, const uint8_t *p,
                                 const uint8_t *end) {
    const size_t len = (size_t)(end - p);
    int64_t r;
    switch (a->accel_type) {
    case ACCEL_VERM:
    case ACCEL_VERM_NOCASE:
        r = vsa_verm_find(0, a->verm.c, 0, 0, 0, a->accel_type == ACCEL_VERM_NOCASE, p, len);
        break;
    case ACCEL_DVERM:
    case ACCEL_DVERM_NOCASE:
        r = vsa_verm_find(4, a->dverm.c1, a->dverm.c2, 0, 0,
                          a->accel_type == ACCEL_DVERM_NOCASE, p, len);
        break;
    case ACCEL_SHUFTI:
        r = vsa_shufti_find(a->shufti.lo.b, a->shufti.hi.b, p, len, 0);
        break;
    case ACCEL_TRUFFLE:
        r = vsa_truffle_find(a->truffle.mask1.b, a->truffle.mask2.b, p, len, 0);
        break;
    default:
        return p;
    }
    return r < 0 ? p : p + r; /* device failure: no skip (the scan reports it) */
}

/* do_accel_block hwlm.c:85-105 */
static size_t hwlm_accel_block(const union AccelAux *aa, const uint8_t *buf, size_t len,
                               size_t start) {
    if (len - start < 16) return start;
    const uint8_t *ptr = hwlm_accel(aa, buf + start, buf + len);
    if (aa->generic.offset) {
        ptr -= aa->generic.offset;
        if (ptr < buf) ptr = buf;
    }
    return (size_t)(ptr - buf);
}

/* do_accel_streaming hwlm.c:114-175 */
static size_t hwlm_accel_stream(const union AccelAux *aux, const uint8_t *hbuf, size_t hlen,
                                const uint8_t *buf, size_t len, size_t start) {
    if (aux->accel_type == ACCEL_NONE || len - start < 16) return start;
    const uint8_t offset = aux->generic.offset;
    if (!start && hlen) {
        const uint8_t *ptr1 = hbuf, *end1 = hbuf + hlen;
        if (hlen >= 16) ptr1 = hwlm_accel(aux, ptr1, end1);
        const bool inaccurate =
            aux->accel_type == ACCEL_DVERM_NOCASE || aux->accel_type == ACCEL_DVERM;
        if ((hlen <= 16 || inaccurate) && end1 != ptr1 && end1 - ptr1 <= 16) {
            uint8_t temp[17];
            const ptrdiff_t tlen = end1 - ptr1;
            memcpy(temp, ptr1, (size_t)tlen);
            memset(temp + tlen, 0, 17 - (size_t)tlen);
            if (len) temp[tlen] = *buf;
            const uint8_t *tp = hwlm_accel(aux, temp, temp + 17);
            if (tp - temp >= tlen) ptr1 = end1;
        }
        if (ptr1 != end1) return start;
    }
    const uint8_t *ptr2 = buf + start;
    const uint8_t *found = hwlm_accel(aux, ptr2, buf + len);
    if (found >= ptr2 + offset) start += (size_t)(found - offset - ptr2);
    return start;
}

/* --------------------------------------------------- drop-in literal -- */

hwlm_error_t hwlmExec(const struct HWLM *tab, const uint8_t *buf, size_t len, size_t start,
                      HWLMCallback cb, struct hs_scratch *scratch, hwlm_group_t groups) {
    if (!tab) return HWLM_ERROR_UNKNOWN;
    if (!groups) return HWLM_SUCCESS;
    if (start >= len) return HWLM_SUCCESS;
    vsa_db *db = registry_get(tab, -1);
    if (!db) return HWLM_ERROR_UNKNOWN;
    std::vector<uint64_t> keys;
    std::vector<uint32_t> ids;
    if (db->type == HWLM_ENGINE_NOOD) {
        if (scan_host(db, buf, len, start, keys, ids) != VSA_OK) return HWLM_ERROR_UNKNOWN;
        return replay_nood(keys.data(), ids.data(), keys.size(), cb, scratch);
    }
    /* accel pre-skip (hwlm.c:85-105, 191-201) on the GPU, on the same
     * upload as the literal scan */
    const HWLM *h = (const HWLM *)db->hblob;
    const union AccelAux *aa = &h->accel0;
    if ((groups & ~h->accel1_groups) == 0) aa = &h->accel1;
    if (aa->accel_type != ACCEL_NONE && len - start >= 16) {
        vsa_ctx *c = db->ctx;
        if (ensure_in(c, 2 * len + 48) != VSA_OK ||
            hipMemcpyAsync(c->ws.d_in, buf, len, hipMemcpyHostToDevice, c->stream) != hipSuccess)
            return HWLM_ERROR_UNKNOWN;
        c->res_host = buf;
        c->res_len = len;
        start = hwlm_accel_block(aa, buf, len, start);
    }
    if (start >= len) {
        db->ctx->res_host = nullptr;
        return HWLM_SUCCESS;
    }
    const int sr = scan_host(db, buf, len, start, keys, ids);
    db->ctx->res_host = nullptr;
    if (sr != VSA_OK) return HWLM_ERROR_UNKNOWN;
    std::vector<vsa::FloodEvent> ev;
    return replay_lit(db, keys.data(), keys.size(), cb, scratch, groups,
                      floods_for(db, buf, len, start, ev));
}

hwlm_error_t fdrExec(const struct FDR *fdr, const uint8_t *buf, size_t len, size_t start,
                     HWLMCallback cb, struct hs_scratch *scratch, hwlm_group_t groups) {
    if (!fdr) return HWLM_ERROR_UNKNOWN;
    if (start >= len) return HWLM_SUCCESS;
    vsa_db *db = registry_get(fdr, HWLM_ENGINE_FDR);
    if (!db) return HWLM_ERROR_UNKNOWN;
    std::vector<uint64_t> keys;
    std::vector<uint32_t> ids;
    if (scan_host(db, buf, len, start, keys, ids) != VSA_OK) return HWLM_ERROR_UNKNOWN;
    std::vector<vsa::FloodEvent> ev;
    return replay_lit(db, keys.data(), keys.size(), cb, scratch, groups,
                      floods_for(db, buf, len, start, ev));
}

hwlm_error_t noodExec(const struct noodTable *n, const uint8_t *buf, size_t len, size_t start,
                      HWLMCallback cb, struct hs_scratch *scratch) {
    if (!n) return HWLM_ERROR_UNKNOWN;
    if (start >= len) return HWLM_SUCCESS;
    vsa_db *db = registry_get(n, HWLM_ENGINE_NOOD);
    if (!db) return HWLM_ERROR_UNKNOWN;
    std::vector<uint64_t> keys;
    std::vector<uint32_t> ids;
    if (scan_host(db, buf, len, start, keys, ids) != VSA_OK) return HWLM_ERROR_UNKNOWN;
    return replay_nood(keys.data(), ids.data(), keys.size(), cb, scratch);
}

/* ------------------------------------------------ drop-in streaming -- */

/* fdrExecStreaming fdr.c:827-855.  len_history 0 scans as block mode (the
 * reference then applies fdr->start and never confirms into history). */
hwlm_error_t fdrExecStreaming(const struct FDR *fdr, const uint8_t *hbuf, size_t hlen,
                              const uint8_t *buf, size_t len, size_t start, HWLMCallback cb,
                              struct hs_scratch *scratch, hwlm_group_t groups) {
    if (!fdr) return HWLM_ERROR_UNKNOWN;
    if (start >= len) return HWLM_SUCCESS;
    vsa_db *db = registry_get(fdr, HWLM_ENGINE_FDR);
    if (!db) return HWLM_ERROR_UNKNOWN;
    std::vector<uint64_t> keys;
    std::vector<uint32_t> ids;
    if (scan_host(db, buf, len, start, keys, ids, hlen ? hbuf + hlen : nullptr, hlen) != VSA_OK)
        return HWLM_ERROR_UNKNOWN;
    std::vector<vsa::FloodEvent> ev;
    return replay_lit(db, keys.data(), keys.size(), cb, scratch, groups,
                      floods_for(db, buf, len, start, ev));
}

/* noodExecStreaming noodle_engine.cpp:136-185 */
hwlm_error_t noodExecStreaming(const struct noodTable *n, const uint8_t *hbuf, size_t hlen,
                               const uint8_t *buf, size_t len, HWLMCallback cb,
                               struct hs_scratch *scratch) {
    if (!n) return HWLM_ERROR_UNKNOWN;
    if (len + hlen < n->msk_len || !len) return HWLM_SUCCESS;
    vsa_db *db = registry_get(n, HWLM_ENGINE_NOOD);
    if (!db) return HWLM_ERROR_UNKNOWN;
    std::vector<uint64_t> keys;
    std::vector<uint32_t> ids;
    if (scan_host(db, buf, len, 0, keys, ids, hlen ? hbuf + hlen : nullptr, hlen) != VSA_OK)
        return HWLM_ERROR_UNKNOWN;
    return replay_nood(keys.data(), ids.data(), keys.size(), cb, scratch);
}

/* hwlmExecStreaming hwlm.c:207-247: buffers from scratch->core_info */
hwlm_error_t hwlmExecStreaming(const struct HWLM *tab, size_t len, size_t start,
                               HWLMCallback cb, struct hs_scratch *scratch,
                               hwlm_group_t groups) {
    if (!tab || !scratch) return HWLM_ERROR_UNKNOWN;
    if (!groups) return HWLM_SUCCESS;
    const char *sc = (const char *)scratch;
    const uint8_t *buf, *hbuf;
    size_t hlen;
    memcpy(&buf, sc + g_core_buf_off.load(), sizeof(buf));
    memcpy(&hbuf, sc + g_core_hbuf_off.load(), sizeof(hbuf));
    memcpy(&hlen, sc + g_core_hlen_off.load(), sizeof(hlen));
    const HWLM *h = (const HWLM *)tab;
    const uint8_t *eng = (const uint8_t *)tab + VSA_ROUNDUP_CL(sizeof(HWLM));
    if (h->type == HWLM_ENGINE_NOOD) {
        if (start) return noodExec((const noodTable *)eng, buf, len, start, cb, scratch);
        return noodExecStreaming((const noodTable *)eng, hbuf, hlen, buf, len, cb, scratch);
    }
    const union AccelAux *aa = &h->accel0;
    if ((groups & ~h->accel1_groups) == 0) aa = &h->accel1;
    start = hwlm_accel_stream(aa, hbuf, hlen, buf, len, start);
    return fdrExecStreaming((const FDR *)eng, hbuf, hlen, buf, len, start, cb, scratch, groups);
}

/* The same entry points under vsa_gpu_* names, for an integration that
 * keeps the reference's own definitions and routes each call by length
 * (the CPU below the measured break-even, the GPU
 * above it). */
hwlm_error_t vsa_gpu_hwlmExec(const struct HWLM *tab, const uint8_t *buf, size_t len,
                              size_t start, HWLMCallback cb, struct hs_scratch *scratch,
                              hwlm_group_t groups) {
    return hwlmExec(tab, buf, len, start, cb, scratch, groups);
}
hwlm_error_t vsa_gpu_hwlmExecStreaming(const struct HWLM *tab, size_t len, size_t start,
                                       HWLMCallback cb, struct hs_scratch *scratch,
                                       hwlm_group_t groups) {
    return hwlmExecStreaming(tab, len, start, cb, scratch, groups);
}
hwlm_error_t vsa_gpu_fdrExec(const struct FDR *fdr, const uint8_t *buf, size_t len,
                             size_t start, HWLMCallback cb, struct hs_scratch *scratch,
                             hwlm_group_t groups) {
    return fdrExec(fdr, buf, len, start, cb, scratch, groups);
}
hwlm_error_t vsa_gpu_noodExec(const struct noodTable *n, const uint8_t *buf, size_t len,
                              size_t start, HWLMCallback cb, struct hs_scratch *scratch) {
    return noodExec(n, buf, len, start, cb, scratch);
}


} // extern "C"

/* The writes of one logical stream (hs_scan: one block-mode write;
 * hs_scan_vector: all pieces) scanned in ONE launch: the history bytes and
 * the writes laid end to end in the context's input buffer, each write a
 * block whose history is what precedes it (<= 16 bytes, enough for the
 * 8-byte HWLM literals); then each write's records replayed in order with
 * its own flood events and ends relative to it.  cbctx is an opaque
 * callback context (no Rose scratch: no INCLUDED_JUMP squash). */
namespace vsa {
/* the host copy of a loaded database's HWLM blob (vsa_internal.h) */
int ctxDevice(const struct vsa_ctx *c) { return c ? c->device : 0; }
int dbHostBlob(const struct vsa_db *db, const uint8_t **blob, size_t *size) {
    if (!db || !blob || !size) return VSA_E_INVALID;
    *blob = db->hblob;
    *size = db->size;
    return VSA_OK;
}
hwlm_error_t exec_pieces(vsa_ctx *c, const vsa_db *db, const u8 *hist, size_t hist_len,
                         const u8 *const *bufs, const size_t *lens, size_t n,
                         LitCallback cb, void *cbctx, void (*on_piece)(void *, size_t)) {
    if (!c || !db) return HWLM_ERROR_UNKNOWN;
    size_t total = 0;
    for (size_t i = 0; i < n; i++) total += lens[i];
    if (!total) return HWLM_SUCCESS;
    const size_t pre = 16, hl0 = std::min<size_t>(hist_len, 16);
    if (ensure_in(c, pre + total + 16) != VSA_OK) return HWLM_ERROR_UNKNOWN;
    /* the history and every piece staged in pinned memory, one DMA (past
     * PIN_STAGE_MAX: a copy per piece) */
    const bool staged = pre + total <= PIN_STAGE_MAX && ensure_hin(c, pre + total) == VSA_OK;
    if (staged) {
        if (hl0) memcpy(c->ws.h_in + pre - hl0, hist + hist_len - hl0, hl0);
    } else if (hl0 && hipMemcpyAsync(c->ws.d_in + pre - hl0, hist + hist_len - hl0, hl0,
                                     hipMemcpyHostToDevice, c->stream) != hipSuccess) {
        return HWLM_ERROR_UNKNOWN;
    }
    std::vector<uint64_t> off, len, st, hl;
    std::vector<size_t> which;
    size_t pos = pre, seen = hist_len;
    for (size_t i = 0; i < n; i++) {
        if (!lens[i]) continue;
        if (staged) {
            memcpy(c->ws.h_in + pos, bufs[i], lens[i]);
        } else if (hipMemcpyAsync(c->ws.d_in + pos, bufs[i], lens[i], hipMemcpyHostToDevice,
                                  c->stream) != hipSuccess) {
            return HWLM_ERROR_UNKNOWN;
        }
        off.push_back(pos);
        len.push_back(lens[i]);
        st.push_back(0);
        hl.push_back(std::min<size_t>(seen, 16));
        which.push_back(i);
        pos += lens[i];
        seen += lens[i];
    }
    if (staged && hipMemcpyAsync(c->ws.d_in + pre - hl0, c->ws.h_in + pre - hl0,
                                 pos - (pre - hl0), hipMemcpyHostToDevice,
                                 c->stream) != hipSuccess)
        return HWLM_ERROR_UNKNOWN;
    uint64_t nm = 0;
    if (scan_blocks_impl(c, db, c->ws.d_in, off.data(), len.data(), st.data(),
                         (uint32_t)off.size(), SCAN_HOST_SORT_SMALL, &nm, hl.data()) != VSA_OK)
        return HWLM_ERROR_UNKNOWN;
    std::vector<uint64_t> keys;
    std::vector<uint32_t> ids;
    if (fetch_records(c, nm, keys, ids) != VSA_OK) return HWLM_ERROR_UNKNOWN;
    hs_scratch *sc = (hs_scratch *)cbctx;
    std::vector<vsa::FloodEvent> ev;
    uint64_t k = 0;
    for (size_t b = 0; b < off.size(); b++) {
        const uint64_t hi = off[b] + len[b];
        uint64_t k2 = k;
        while (k2 < nm && (keys[k2] >> VSA_KEY_END_SHIFT) < hi) {
            keys[k2] -= off[b] << VSA_KEY_END_SHIFT; /* end relative to the write */
            k2++;
        }
        if (on_piece) on_piece(cbctx, which[b]);
        hwlm_error_t r;
        if (db->type == HWLM_ENGINE_NOOD) {
            r = replay_nood(keys.data() + k, ids.data() + k, k2 - k, cb, sc);
        } else {
            r = replay_lit(db, keys.data() + k, k2 - k, cb, sc, HWLM_ALL_GROUPS,
                           floods_for(db, bufs[which[b]], len[b], 0, ev), false);
        }
        if (r != HWLM_SUCCESS) return r;
        k = k2;
    }
    return HWLM_SUCCESS;
}
/* One launch over device-resident blocks (hlens NULL: block mode) and the
 * sorted records copied to the host (want_records) or only counted. */
int scan_records(vsa_ctx *c, const vsa_db *db, const u8 *d_data, const uint64_t *offsets,
                 const uint64_t *lens, const uint64_t *hlens, uint32_t nblocks,
                 std::vector<uint64_t> *keys, std::vector<uint32_t> *ids, uint64_t *n_out,
                 const vsa_plan *plan) {
    uint64_t nm = 0;
    int r;
    if (plan) {
        r = vsa_scan_plan(c, db, plan, 0, &nm);
    } else {
        std::vector<uint64_t> st(nblocks, 0);
        r = scan_blocks_impl(c, db, d_data, offsets, lens, st.data(), nblocks, 0, &nm, hlens);
    }
    if (r != VSA_OK) return r;
    *n_out = nm;
    if (!keys) return VSA_OK;
    keys->resize(nm);
    ids->resize(nm);
    if (nm) {
        VSA_CHECK(hipMemcpyAsync(keys->data(), c->ws.d_keys[c->cur], nm * 8,
                                 hipMemcpyDeviceToHost, c->stream));
        VSA_CHECK(hipMemcpyAsync(ids->data(), c->ws.d_ids[c->cur], nm * 4,
                                 hipMemcpyDeviceToHost, c->stream));
        VSA_CHECK(hipStreamSynchronize(c->stream));
    }
    return VSA_OK;
}

int records_mark(vsa_ctx *c) {
    if (!c->ev_mark) VSA_CHECK(hipEventCreateWithFlags(&c->ev_mark, hipEventDisableTiming));
    VSA_CHECK(hipEventRecord(c->ev_mark, c->stream));
    c->marked = true;
    return VSA_OK;
}

int records_fetch_async(vsa_ctx *c, uint64_t n, uint64_t *h_keys, uint32_t *h_ids,
                        bool remark) {
    if (!c->ev_rec) VSA_CHECK(hipEventCreateWithFlags(&c->ev_rec, hipEventDisableTiming));
    if (!c->copy_stream) {
        VSA_CHECK(hipSetDevice(c->device));
        VSA_CHECK(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    }
    /* the copy starts when the scan that made the records has ended: its
     * mark, or (no mark, or a rescan since) everything queued so far */
    if (!c->marked || remark) VSA_CHECK(records_mark(c) == VSA_OK ? hipSuccess : hipErrorUnknown);
    c->marked = false;
    VSA_CHECK(hipStreamWaitEvent(c->copy_stream, c->ev_mark, 0));
    if (n) {
        VSA_CHECK(hipMemcpyAsync(h_keys, c->ws.d_keys[c->cur], n * 8, hipMemcpyDeviceToHost,
                                 c->copy_stream));
        VSA_CHECK(hipMemcpyAsync(h_ids, c->ws.d_ids[c->cur], n * 4, hipMemcpyDeviceToHost,
                                 c->copy_stream));
    }
    VSA_CHECK(hipEventRecord(c->ev_rec, c->copy_stream));
    /* the scan stream's next work (this context's next scan rewrites the
     * records) waits for the copy, on the device */
    VSA_CHECK(hipStreamWaitEvent(c->stream, c->ev_rec, 0));
    return VSA_OK;
}

int records_wait(vsa_ctx *c) {
    if (!c->ev_rec) return VSA_OK;
    /* polled (a blocking wait wakes on a coarse tick, runtime.hip
     * wait_stream): spin ~100 us, then yield; past 50 ms block */
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0;; i++) {
        const hipError_t e = hipEventQuery(c->ev_rec);
        if (e == hipSuccess) return VSA_OK;
        if (e != hipErrorNotReady) VSA_CHECK(e);
        (void)hipGetLastError();
        if ((i & 15) == 15) {
            const auto dt = std::chrono::steady_clock::now() - t0;
            if (dt > std::chrono::milliseconds(50)) {
                VSA_CHECK(hipEventSynchronize(c->ev_rec));
                return VSA_OK;
            }
            if (dt > std::chrono::microseconds(100)) sched_yield();
        }
    }
}

void *host_pinned_alloc(size_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, std::max<size_t>(bytes, 64), hipHostMallocDefault) != hipSuccess)
        return nullptr;
    return p;
}

void host_pinned_free(void *p) {
    if (p) (void)hipHostFree(p);
}

/* The records of one call (ends relative to that call's buffer) through
 * the callback, without flood emulation (no host buffer address) */
int replay_records(const vsa_db *db, const uint64_t *keys, const uint32_t *ids, uint64_t n,
                   LitCallback cb, void *cbctx) {
    hs_scratch *sc = (hs_scratch *)cbctx;
    if (db->type == HWLM_ENGINE_NOOD) return replay_nood(keys, ids, n, cb, sc);
    return replay_lit(db, keys, n, cb, sc, HWLM_ALL_GROUPS, nullptr, false);
}
} // namespace vsa

extern "C" {

void vsa_get_scratch_core_info(long *buf_off, long *hbuf_off, long *hlen_off) {
    *buf_off = g_core_buf_off.load();
    *hbuf_off = g_core_hbuf_off.load();
    *hlen_off = g_core_hlen_off.load();
}

void vsa_set_scratch_core_info(long buf_off, long hbuf_off, long hlen_off) {
    g_core_buf_off.store(buf_off);
    g_core_hbuf_off.store(hbuf_off);
    g_core_hlen_off.store(hlen_off);
}

/* ----------------------------------------------------- drop-in accel -- */

int64_t vsa_shufti_find(const uint8_t lo[16], const uint8_t hi[16], const uint8_t *buf,
                        size_t len, int reverse) {
    uint8_t cls[32];
    cls_from_shufti(lo, hi, cls);
    uint64_t f = len, l = 0;
    if (class_host(cls, nullptr, buf, len, &f, &l) != VSA_OK) return -2;
    return reverse ? (int64_t)l - 1 : (int64_t)f;
}

int64_t vsa_truffle_find(const uint8_t m1[16], const uint8_t m2[16], const uint8_t *buf,
                         size_t len, int reverse) {
    uint8_t cls[32];
    cls_from_truffle(m1, m2, cls);
    uint64_t f = len, l = 0;
    if (class_host(cls, nullptr, buf, len, &f, &l) != VSA_OK) return -2;
    return reverse ? (int64_t)l - 1 : (int64_t)f;
}

int64_t vsa_verm_find(int mode, uint8_t c1, uint8_t c2, uint8_t m1, uint8_t m2, int nocase,
                      const uint8_t *buf, size_t len) {
    uint8_t cls[32], cls2[32];
    uint8_t cm = nocase ? 0xdf : 0xff;
    uint64_t f = len, l = 0;
    switch (mode) {
    case 0: /* vermicelliExec */
    case 2: /* rvermicelliExec */
        cls_from_masked(c1, cm, false, cls);
        break;
    case 1: /* nvermicelliExec */
    case 3: /* rnvermicelliExec */
        cls_from_masked(c1, cm, true, cls);
        break;
    case 4: /* vermicelliDoubleExec */
        cls_from_masked(c1, cm, false, cls);
        cls_from_masked(c2, cm, false, cls2);
        break;
    case 5: /* vermicelliDoubleMaskedExec */
        cls_from_masked(c1, m1, false, cls);
        cls_from_masked(c2, m2, false, cls2);
        break;
    case 6: /* rvermicelliDoubleExec */
        cls_from_masked(c1, cm, false, cls);
        cls_from_masked(c2, cm, false, cls2);
        break;
    default:
        return -2;
    }
    bool pair = mode >= 4;
    if (class_host(cls, pair ? cls2 : nullptr, buf, len, &f, &l) != VSA_OK) return -2;
    if (mode == 2 || mode == 3) return (int64_t)l - 1;
    if (mode == 6) {
        /* vermicelli_simd.cpp:360-423: position of c2 in the last pair (the
         * pair bitmap marks c1's position, so that is `last`); a c2 at
         * buf[0] is a partial pair; else buf - 1 */
        if (l) return (int64_t)l;
        if (len && cls_has(cls2, buf[0])) return 0;
        return -1;
    }
    if (pair && f == len && len && cls_has(cls, buf[len - 1])) {
        /* partial match at the end (vermicelli_simd.cpp:349-355) */
        return (int64_t)len - 1;
    }
    return (int64_t)f;
}

static void m128_bytes(vsa_m128_t m, uint8_t out[16]) { memcpy(out, &m, 16); }

/* The pointer-returning drop-ins have no error channel in the reference
 * ABI.  A device failure (the vsa_*_find helpers return -2) is recorded for
 * vsa_last_error() and answered with the no-skip pointer: buf for forward
 * scans, buf_end - 1 for reverse ones (every accel caller, hwlm.c:48-105 and
 * accel.c:35-180, then scans from there), never buf + (-2). */
static thread_local int t_last_error = VSA_OK;

static void note_error(const char *who) {
    t_last_error = VSA_E_DEVICE;
    if (getenv("VSA_DEBUG")) fprintf(stderr, "vsa: %s: device failure\n", who);
}

static const uint8_t *fwd_result(int64_t r, const uint8_t *buf, const uint8_t *buf_end,
                                 const char *who) {
    if (r == -2) {
        note_error(who);
        return buf;
    }
    return r < 0 ? buf_end : buf + r;
}

static const uint8_t *rev_result(int64_t r, const uint8_t *buf, const uint8_t *buf_end,
                                 const char *who) {
    if (r == -2) {
        note_error(who);
        return buf_end - 1;
    }
    return buf + r; /* -1: buf - 1, "not found" */
}

int vsa_last_error(void) {
    const int e = t_last_error;
    t_last_error = VSA_OK;
    return e;
}

const uint8_t *shuftiExec(vsa_m128_t mask_lo, vsa_m128_t mask_hi, const uint8_t *buf,
                          const uint8_t *buf_end) {
    uint8_t lo[16], hi[16];
    m128_bytes(mask_lo, lo);
    m128_bytes(mask_hi, hi);
    return fwd_result(vsa_shufti_find(lo, hi, buf, (size_t)(buf_end - buf), 0), buf, buf_end,
                      "shuftiExec");
}

void vsa_set_accel_vector_size(uint32_t vsize) {
    if (vsize == 16 || vsize == 32 || vsize == 64) g_vector_size = vsize;
}

int64_t vsa_shufti_double_find(const uint8_t lo1[16], const uint8_t hi1[16],
                               const uint8_t lo2[16], const uint8_t hi2[16],
                               const uint8_t *buf, size_t len) {
    return pair_host(lo1, hi1, lo2, hi2, buf, len, g_vector_size);
}

const uint8_t *shuftiDoubleExec(vsa_m128_t mask1_lo, vsa_m128_t mask1_hi, vsa_m128_t mask2_lo,
                                vsa_m128_t mask2_hi, const uint8_t *buf,
                                const uint8_t *buf_end) {
    uint8_t lo1[16], hi1[16], lo2[16], hi2[16];
    m128_bytes(mask1_lo, lo1);
    m128_bytes(mask1_hi, hi1);
    m128_bytes(mask2_lo, lo2);
    m128_bytes(mask2_hi, hi2);
    return fwd_result(vsa_shufti_double_find(lo1, hi1, lo2, hi2, buf, (size_t)(buf_end - buf)),
                      buf, buf_end, "shuftiDoubleExec");
}

int vsa_shufti_build_double_masks(const uint8_t onechar[32], const uint8_t *pairs,
                                  size_t npairs, uint8_t lo1[16], uint8_t hi1[16],
                                  uint8_t lo2[16], uint8_t hi2[16]) {
    return vsa::shuftiDoubleMasks(onechar, pairs, npairs, lo1, hi1, lo2, hi2) ? 0 : -1;
}

const uint8_t *rshuftiExec(vsa_m128_t mask_lo, vsa_m128_t mask_hi, const uint8_t *buf,
                           const uint8_t *buf_end) {
    uint8_t lo[16], hi[16];
    m128_bytes(mask_lo, lo);
    m128_bytes(mask_hi, hi);
    return rev_result(vsa_shufti_find(lo, hi, buf, (size_t)(buf_end - buf), 1), buf, buf_end,
                      "rshuftiExec");
}

const uint8_t *truffleExec(vsa_m128_t mask1, vsa_m128_t mask2, const uint8_t *buf,
                           const uint8_t *buf_end) {
    uint8_t a[16], b[16];
    m128_bytes(mask1, a);
    m128_bytes(mask2, b);
    return fwd_result(vsa_truffle_find(a, b, buf, (size_t)(buf_end - buf), 0), buf, buf_end,
                      "truffleExec");
}

const uint8_t *rtruffleExec(vsa_m128_t mask1, vsa_m128_t mask2, const uint8_t *buf,
                            const uint8_t *buf_end) {
    uint8_t a[16], b[16];
    m128_bytes(mask1, a);
    m128_bytes(mask2, b);
    return rev_result(vsa_truffle_find(a, b, buf, (size_t)(buf_end - buf), 1), buf, buf_end,
                      "rtruffleExec");
}

static const uint8_t *verm_fwd(int mode, char c1, char c2, char m1, char m2, char nocase,
                               const uint8_t *buf, const uint8_t *buf_end, const char *who) {
    return fwd_result(vsa_verm_find(mode, (uint8_t)c1, (uint8_t)c2, (uint8_t)m1, (uint8_t)m2,
                                    nocase, buf, (size_t)(buf_end - buf)),
                      buf, buf_end, who);
}

static const uint8_t *verm_rev(int mode, char c1, char c2, char nocase, const uint8_t *buf,
                               const uint8_t *buf_end, const char *who) {
    return rev_result(vsa_verm_find(mode, (uint8_t)c1, (uint8_t)c2, 0, 0, nocase, buf,
                                    (size_t)(buf_end - buf)),
                      buf, buf_end, who);
}

const uint8_t *vermicelliExec(char c, char nocase, const uint8_t *buf, const uint8_t *buf_end) {
    return verm_fwd(0, c, 0, 0, 0, nocase, buf, buf_end, "vermicelliExec");
}
const uint8_t *nvermicelliExec(char c, char nocase, const uint8_t *buf, const uint8_t *buf_end) {
    return verm_fwd(1, c, 0, 0, 0, nocase, buf, buf_end, "nvermicelliExec");
}
const uint8_t *rvermicelliExec(char c, char nocase, const uint8_t *buf, const uint8_t *buf_end) {
    return verm_rev(2, c, 0, nocase, buf, buf_end, "rvermicelliExec");
}
const uint8_t *rnvermicelliExec(char c, char nocase, const uint8_t *buf,
                                const uint8_t *buf_end) {
    return verm_rev(3, c, 0, nocase, buf, buf_end, "rnvermicelliExec");
}
const uint8_t *vermicelliDoubleExec(char c1, char c2, char nocase, const uint8_t *buf,
                                    const uint8_t *buf_end) {
    return verm_fwd(4, c1, c2, 0, 0, nocase, buf, buf_end, "vermicelliDoubleExec");
}
const uint8_t *rvermicelliDoubleExec(char c1, char c2, char nocase, const uint8_t *buf,
                                     const uint8_t *buf_end) {
    return verm_rev(6, c1, c2, nocase, buf, buf_end, "rvermicelliDoubleExec");
}

const uint8_t *vermicelliDoubleMaskedExec(char c1, char c2, char m1, char m2,
                                          const uint8_t *buf, const uint8_t *buf_end) {
    return verm_fwd(5, c1, c2, m1, m2, 0, buf, buf_end, "vermicelliDoubleMaskedExec");
}

/* accel.c:35-180 dispatch for the forward schemes HWLM and NFAs use */
/* accel.c:36-183: minimum lengths (16, 17 for the double forms, which stop
 * one byte early), then rv = MAX(c + offset, rv) - offset. */
const uint8_t *run_accel(const union AccelAux *accel, const uint8_t *c, const uint8_t *c_end) {
    const size_t len = (size_t)(c_end - c);
    int64_t r;
    switch (accel->accel_type) {
    case ACCEL_NONE:
        return c;
    case ACCEL_VERM:
    case ACCEL_VERM_NOCASE:
        if (c + 15 >= c_end) return c;
        r = vsa_verm_find(0, accel->verm.c, 0, 0, 0, accel->accel_type == ACCEL_VERM_NOCASE, c,
                          len);
        break;
    case ACCEL_DVERM:
    case ACCEL_DVERM_NOCASE:
        if (c + 16 + 1 >= c_end) return c;
        r = vsa_verm_find(4, accel->dverm.c1, accel->dverm.c2, 0, 0,
                          accel->accel_type == ACCEL_DVERM_NOCASE, c, len - 1);
        break;
    case ACCEL_DVERM_MASKED:
        if (c + 16 + 1 >= c_end) return c;
        r = vsa_verm_find(5, accel->dverm.c1, accel->dverm.c2, accel->dverm.m1, accel->dverm.m2,
                          0, c, len - 1);
        break;
    case ACCEL_SHUFTI:
        if (c + 15 >= c_end) return c;
        r = vsa_shufti_find(accel->shufti.lo.b, accel->shufti.hi.b, c, len, 0);
        break;
    case ACCEL_TRUFFLE:
        if (c + 15 >= c_end) return c;
        r = vsa_truffle_find(accel->truffle.mask1.b, accel->truffle.mask2.b, c, len, 0);
        break;
    case ACCEL_DSHUFTI:
        if (c + 15 + 1 >= c_end) return c;
        r = vsa_shufti_double_find(accel->dshufti.lo1.b, accel->dshufti.hi1.b,
                                   accel->dshufti.lo2.b, accel->dshufti.hi2.b, c, len - 1);
        break;
    case ACCEL_RED_TAPE:
        r = (int64_t)len;
        break;
    default:
        return c;
    }
    if (r < 0) { /* device failure: no acceleration (see fwd_result) */
        note_error("run_accel");
        return c;
    }
    const uint8_t *rv = c + r;
    rv = std::max(c + accel->generic.offset, rv);
    return rv - accel->generic.offset;
}

int vsa_hwlm_register(const void *blob, int bare_type) {
    if (!blob) return VSA_E_INVALID;
    const uint8_t *p = (const uint8_t *)blob;
    size_t size;
    if (bare_type < 0) {
        size = VSA_ROUNDUP_CL(sizeof(HWLM)) +
               engine_size(p + VSA_ROUNDUP_CL(sizeof(HWLM)), p[0]);
    } else {
        if (bare_type != HWLM_ENGINE_NOOD && bare_type != HWLM_ENGINE_FDR) return VSA_E_INVALID;
        size = engine_size(p, bare_type);
    }
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_registered[blob] = size;
    return VSA_OK;
}

int vsa_hwlm_unregister(const void *blob) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    return g_registered.erase(blob) ? VSA_OK : VSA_E_INVALID;
}

void vsa_set_scratch_layout(long fdr_conf_off, long fdr_conf_offset_off) {
    g_fdr_conf_off.store(fdr_conf_off);
    g_fdr_conf_offset_off.store(fdr_conf_offset_off);
}

void vsa_get_scratch_layout(long *fdr_conf_off, long *fdr_conf_offset_off) {
    *fdr_conf_off = g_fdr_conf_off.load();
    *fdr_conf_offset_off = g_fdr_conf_offset_off.load();
}

/* ---------------------------------------------------------- builder --- */

void vsa_build_opts_default(vsa_build_opts_t *o) {
    o->engine_hint = -1;
    o->allow_noodle = 1;
    o->allow_teddy = 1;
    o->allow_fat_teddy = 1;
    o->allow_flood = 1; /* the reference Grey default (grey.cpp:68) */
}

int vsa_hwlm_build(const vsa_literal_t *lits, size_t n, const vsa_build_opts_t *opts,
                   void **blob, size_t *size) {
    if (!lits || !n || !blob || !size) return VSA_E_INVALID;
    vsa::BuildOptions bo;
    if (opts) {
        bo.engine_hint = opts->engine_hint;
        bo.allow_noodle = opts->allow_noodle;
        bo.allow_teddy = opts->allow_teddy;
        bo.allow_fat_teddy = opts->allow_fat_teddy;
        bo.allow_flood = opts->allow_flood;
    }
    std::vector<vsa::Literal> v;
    v.reserve(n);
    for (size_t i = 0; i < n; i++) {
        const vsa_literal_t &l = lits[i];
        if (!l.s || !l.len) return VSA_E_INVALID;
        v.push_back(vsa::makeLiteral(l.s, l.len, l.nocase, l.noruns, l.id, l.groups, l.msk,
                                     l.cmp, l.msk_len));
    }
    uint8_t *out = nullptr;
    int r = vsa::buildHwlm(std::move(v), bo, &out, size);
    if (r != VSA_OK) return r;
    *blob = out;
    return VSA_OK;
}

void vsa_blob_free(void *blob) { free(blob); }

int vsa_hwlm_set_accel(void *blob, const union AccelAux *a0, const union AccelAux *a1,
                       uint64_t g1) {
    if (!blob) return VSA_E_INVALID;
    HWLM *h = (HWLM *)blob;
    if (a0) memcpy(&h->accel0, a0, sizeof(*a0));
    if (a1) memcpy(&h->accel1, a1, sizeof(*a1));
    h->accel1_groups = g1;
    return VSA_OK;
}

int vsa_shufti_build_masks(const uint8_t cls[32], uint8_t lo[16], uint8_t hi[16]) {
    return vsa::shuftiMasks(cls, lo, hi);
}

void vsa_truffle_build_masks(const uint8_t cls[32], uint8_t m1[16], uint8_t m2[16]) {
    vsa::truffleMasks(cls, m1, m2);
}


} /* extern "C" */
