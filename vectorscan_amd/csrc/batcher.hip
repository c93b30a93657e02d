/*
 * batcher.hip -- the batching service (vsa_batcher_*): concurrent drop-in
 * calls from many host threads share one launch per window.
 */
#include "runtime_internal.h"

/* ------------------------------------------------- batching service --- */

/* Concurrent drop-in calls (many host threads scanning blocks, each through
 * its Rose floating table: rose/block.c:259, hsbench -T) share launches: a
 * worker thread with its own context takes the calls queued within a short
 * window, stages all their buffers into pinned memory, sends them in one
 * DMA, scans them as the blocks of ONE launch (vsa_scan_blocks, starts per
 * block) and hands each caller its records (rebased to its buffer); the
 * caller replays them through its own callback on its own thread, exactly as
 * hwlmExec does (groups, NOREPEAT, squash, flood events).  A call pays one
 * launch shared by the batch instead of one of its own.  The accel pre-skip
 * is not applied on this path (it only moves `start` past positions where no
 * literal can match). */
struct vsa_batcher {
    struct Req {
        const void *tab;
        const uint8_t *buf;
        size_t len, start;
        vsa_db *db = nullptr;
        std::vector<uint64_t> keys;
        std::vector<uint32_t> ids;
        int rc = VSA_OK;
        bool done = false;
    };
    int device = 0;
    uint32_t max_batch = 256;
    uint32_t window_us = 20;
    size_t max_bytes = 64u << 20;
    std::mutex m;
    std::condition_variable cv_req, cv_done;
    std::deque<Req *> q;
    bool stop = false;
    /* callers inside vsa_batcher_hwlmExec that still hold m or will re-lock
     * it (counted under m); destroy waits for zero before freeing m / cv */
    uint32_t inflight = 0;
    std::condition_variable cv_idle;
    std::thread worker;
    uint64_t batches = 0, calls = 0;

    void run() {
        vsa_ctx *c = nullptr;
        if (vsa_ctx_create(device, &c) != VSA_OK) c = nullptr;
        t_ctx = c; /* registry_get loads the tables on this context */
        std::vector<Req *> batch;
        std::vector<uint64_t> offs, lens, starts;
        std::vector<uint64_t> keys;
        std::vector<uint32_t> ids;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(m);
                cv_req.wait(lk, [&] { return stop || !q.empty(); });
                if (stop && q.empty()) break;
                /* a short window for more callers to join the launch */
                if (q.size() < max_batch && window_us)
                    cv_req.wait_for(lk, std::chrono::microseconds(window_us),
                                    [&] { return stop || q.size() >= max_batch; });
                batch.clear();
                size_t bytes = 0;
                while (!q.empty() && batch.size() < max_batch &&
                       (batch.empty() || bytes + q.front()->len <= max_bytes)) {
                    bytes += q.front()->len;
                    batch.push_back(q.front());
                    q.pop_front();
                }
            }
            /* one launch per table in the batch */
            std::stable_sort(batch.begin(), batch.end(),
                             [](const Req *a, const Req *b) { return a->tab < b->tab; });
            for (size_t i = 0; i < batch.size();) {
                size_t j = i;
                while (j < batch.size() && batch[j]->tab == batch[i]->tab) j++;
                const int rc = c ? scan_group(c, batch.data() + i, j - i, offs, lens, starts,
                                              keys, ids)
                                 : VSA_E_DEVICE;
                for (size_t k = i; k < j; k++)
                    if (rc != VSA_OK) batch[k]->rc = rc;
                i = j;
            }
            {
                std::lock_guard<std::mutex> lk(m);
                for (Req *r : batch) r->done = true;
                batches++;
                calls += batch.size();
            }
            cv_done.notify_all();
        }
        if (c) {
            while (!t_registry.empty()) vsa_db_free(t_registry.begin()->second);
            vsa_ctx_destroy(c);
        }
        t_ctx = nullptr;
    }

    static int scan_group(vsa_ctx *c, Req **rq, size_t n, std::vector<uint64_t> &offs,
                          std::vector<uint64_t> &lens, std::vector<uint64_t> &starts,
                          std::vector<uint64_t> &keys, std::vector<uint32_t> &ids) {
        vsa_db *db = registry_get(rq[0]->tab, -1);
        if (!db) return VSA_E_INVALID;
        size_t total = 0;
        offs.resize(n);
        lens.resize(n);
        starts.resize(n);
        for (size_t k = 0; k < n; k++) {
            offs[k] = total;
            lens[k] = rq[k]->len;
            starts[k] = rq[k]->start;
            total += rq[k]->len;
        }
        int r;
        if ((r = ensure_in(c, total + 16)) != VSA_OK) return r;
        if ((r = ensure_hin(c, total)) != VSA_OK) return r;
        for (size_t k = 0; k < n; k++) memcpy(c->ws.h_in + offs[k], rq[k]->buf, rq[k]->len);
        c->res_host = nullptr;
        VSA_CHECK(hipMemcpyAsync(c->ws.d_in, c->ws.h_in, total, hipMemcpyHostToDevice, c->stream));
        uint64_t nm = 0;
        if ((r = scan_blocks_impl(c, db, c->ws.d_in, offs.data(), lens.data(), starts.data(),
                                  (uint32_t)n, 0, &nm)) != VSA_OK)
            return r;
        if ((r = fetch_records(c, nm, keys, ids)) != VSA_OK) return r;
        /* the records are in end order: each caller's are one run */
        uint64_t k0 = 0;
        for (size_t k = 0; k < n; k++) {
            const uint64_t hi = (offs[k] + lens[k]) << VSA_KEY_END_SHIFT;
            uint64_t k1 = k0;
            while (k1 < nm && keys[k1] < hi) k1++;
            Req *q = rq[k];
            q->db = db;
            q->keys.resize(k1 - k0);
            q->ids.assign(ids.begin() + (ptrdiff_t)k0, ids.begin() + (ptrdiff_t)k1);
            const uint64_t base = offs[k] << VSA_KEY_END_SHIFT;
            for (uint64_t i = k0; i < k1; i++) q->keys[i - k0] = keys[i] - base;
            k0 = k1;
        }
        return VSA_OK;
    }
};

extern "C" {

int vsa_batcher_create(int device, uint32_t max_batch, uint32_t window_us, vsa_batcher_t **out) {
    if (!out || !max_batch || max_batch > VSA_MAX_BLOCKS) return VSA_E_INVALID;
    vsa_batcher *b = new (std::nothrow) vsa_batcher;
    if (!b) return VSA_E_NOMEM;
    b->device = device;
    b->max_batch = max_batch;
    b->window_us = window_us;
    b->worker = std::thread([b] { b->run(); });
    *out = b;
    return VSA_OK;
}

int vsa_batcher_destroy(vsa_batcher_t *b) {
    if (!b) return VSA_E_INVALID;
    {
        std::lock_guard<std::mutex> lk(b->m);
        b->stop = true;
    }
    b->cv_req.notify_all();
    b->worker.join();
    {
        /* the worker finished every queued call before exiting; wait for
         * their callers to leave the mutex (a woken caller re-locks it) */
        std::unique_lock<std::mutex> lk(b->m);
        b->cv_idle.wait(lk, [&] { return b->inflight == 0; });
    }
    delete b;
    return VSA_OK;
}

int vsa_batcher_stats(vsa_batcher_t *b, uint64_t *batches, uint64_t *calls) {
    if (!b) return VSA_E_INVALID;
    std::lock_guard<std::mutex> lk(b->m);
    if (batches) *batches = b->batches;
    if (calls) *calls = b->calls;
    return VSA_OK;
}

hwlm_error_t vsa_batcher_hwlmExec(vsa_batcher_t *b, const struct HWLM *tab, const uint8_t *buf,
                                  size_t len, size_t start, HWLMCallback cb,
                                  struct hs_scratch *scratch, hwlm_group_t groups) {
    if (!b || !tab) return HWLM_ERROR_UNKNOWN;
    if (!groups || start >= len) return HWLM_SUCCESS;
    /* a buffer that would fill a batch on its own goes alone */
    if (len > b->max_bytes / 4) return hwlmExec(tab, buf, len, start, cb, scratch, groups);
    vsa_batcher::Req r;
    r.tab = tab;
    r.buf = buf;
    r.len = len;
    r.start = start;
    {
        /* destroy may run concurrently: a call that finds it stopping is
         * refused; one already queued is served (the worker drains the
         * queue before it exits) and is counted until it has left m */
        std::unique_lock<std::mutex> lk(b->m);
        if (b->stop) return HWLM_ERROR_UNKNOWN;
        b->inflight++;
        b->q.push_back(&r);
        b->cv_req.notify_one();
        b->cv_done.wait(lk, [&] { return r.done; });
        if (--b->inflight == 0 && b->stop) b->cv_idle.notify_all();
    }
    if (r.rc != VSA_OK || !r.db) return HWLM_ERROR_UNKNOWN;
    if (r.db->type == HWLM_ENGINE_NOOD)
        return replay_nood(r.keys.data(), r.ids.data(), r.keys.size(), cb, scratch);
    std::vector<vsa::FloodEvent> ev;
    return replay_lit(r.db, r.keys.data(), r.keys.size(), cb, scratch, groups,
                      floods_for(r.db, buf, len, start, ev));
}

} /* extern "C" */
