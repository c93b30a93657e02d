/*
 * hs_lit.cpp — pure-literal databases: hs_compile_lit_multi, hs_scan,
 * hs_scan_vector and streams (include/vectorscan_amd_hs.h) over the GPU
 * HWLM scan (runtime.hip vsa::exec_pieces: one launch per call).
 *
 * Compile — what the reference's build does for pure literals
 * (compiler.cpp:391-433 addLitExpression, :121-150 ParsedLitExpression,
 * ng.cpp:578-625 NG::addLiteral, rose_build_matchers.cpp:700-743
 * addFragmentLiteral):
 *   - a caseless pattern is a ue2_literal with every position nocase
 *     (ue2_literal::push_back upper-cases and marks it), so its HWLM
 *     literal is nocase;
 *   - patterns with the same literal tail and case share one fragment; the
 *     fragment's HWLM literal is the last ROSE_SHORT_LITERAL_LEN_MAX = 8
 *     bytes, the rest of a longer literal is checked when the tail matches
 *     (CHECK_LONG_LIT / CHECK_MED_LIT);
 *   - NOREPEAT only where every pattern of the fragment is <= 8 bytes and
 *     single-match (isNoRunsLiteral :511-557);
 *   - ids: SINGLEMATCH must agree across patterns of one id
 *     (report_manager.cpp:212-236); one exhaustion key per single-match id.
 * Run — pureLiteralBlockExec (runtime.c:204-230) / pureLiteralStreamExec
 * (:802-831) with roseCallback (match.c): an HWLM end e in a write at stream
 * offset o is `to` = o + e + 1 (lit_offset_adjust = offset + 1); each
 * pattern of the fragment, in compile order, reports unless its long-literal
 * check fails, its id is exhausted, or its id was already reported at this
 * `to` (dedupe keys are per external id); from = to - len under
 * HS_FLAG_SOM_LEFTMOST (makeSomRelativeCallback), else 0.  The SOM reports
 * of an id with several patterns go through the SOM dedupe log instead: the
 * leftmost start per id at one offset, delivered when the offset moves on
 * or the write ends (flushStoredSomMatches).  A nonzero
 * callback return ends the scan: HS_SCAN_TERMINATED, and a terminated
 * stream stays terminated (runtime.c:883-893).
 */
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "vectorscan_amd.h"
#include "vectorscan_amd_hs.h"
#include "vsa_internal.h"

namespace {

constexpr uint32_t DB_MAGIC = 0x56534c44u;      /* "VSLD" */
constexpr uint32_t SCRATCH_MAGIC = 0x56534c53u; /* "VSLS" */
constexpr uint32_t STREAM_MAGIC = 0x5653534du;  /* "VSSM" */
constexpr size_t SHORT_LIT = 8;                 /* ROSE_SHORT_LITERAL_LEN_MAX */
constexpr size_t HIST_MIN = 16;                 /* history handed to the GPU */
constexpr size_t LIMIT_PATTERN_LENGTH = 16000;  /* grey.cpp:148 */
constexpr unsigned LIMIT_PATTERN_COUNT = 8000000; /* grey.cpp:147 */
constexpr uint32_t NO_EKEY = ~0u;
constexpr int KEY_END_SHIFT = 24; /* vsa_match_t.key: end << 24 */

std::atomic<uint64_t> g_serial{1};

struct Pattern {
    uint32_t id = 0;
    uint32_t ekey = NO_EKEY; /* exhaustion key (single-match ids) */
    bool som = false;
    bool som_dedupe = false; /* SOM report of an id with several patterns */
    bool caseless = false;
    std::string s; /* as compiled: upper-cased when caseless */
};

inline uint8_t upper(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }

} // namespace

struct vsa_hs_database {
    uint32_t magic = DB_MAGIC;
    uint32_t mode = 0;
    uint64_t serial = 0;
    uint8_t *hwlm = nullptr;
    size_t hwlm_size = 0;
    std::vector<Pattern> pats;
    std::vector<std::vector<uint32_t>> frags; /* fragment -> patterns */
    uint32_t n_ekeys = 0;
    uint32_t min_width = 0;
    size_t max_len = 0;
    bool dedupe = false; /* some id belongs to more than one pattern */
    bool simple = false; /* one report per HWLM record (see vsa_hs_scan_corpus) */
    /* the compile inputs, as given (the serialized form, which
     * vsa_hs_deserialize_database compiles again) */
    unsigned mode_full = 0;
    struct Src {
        std::string e;
        unsigned flags, id;
    };
    std::vector<Src> src;
};

struct vsa_hs_scratch {
    uint32_t magic = SCRATCH_MAGIC;
    std::atomic<bool> in_use{false};
    vsa_ctx_t *ctx = nullptr;
    std::vector<std::pair<uint64_t, vsa_db_t *>> dbs; /* serial -> device copy */
};

/* per-stream state: stream offset, the last bytes written (history), the
 * exhaustion vector and the terminated status */
struct vsa_hs_stream {
    uint32_t magic = STREAM_MAGIC;
    const vsa_hs_database *db = nullptr;
    uint64_t offset = 0;
    std::vector<uint8_t> hist;
    std::vector<uint8_t> exhausted;
    bool terminated = false;
};

namespace {

vsa_hs_compile_error_t *make_error(const std::string &msg, int expression) {
    vsa_hs_compile_error_t *e = (vsa_hs_compile_error_t *)malloc(sizeof(*e));
    if (!e) return nullptr;
    e->message = strdup(msg.c_str());
    e->expression = expression;
    return e;
}

bool valid_db(const vsa_hs_database_t *db) { return db && db->magic == DB_MAGIC; }

/* Persistent workers for the corpus replay: starting 16 threads per call
 * cost as much as the replay itself.  run(T, fn) runs fn(1..T-1) on the
 * workers and fn(0) on the caller, and returns when all are done.  One job
 * at a time (callers serialize on `call`); the pool is never destroyed (its
 * idle threads end with the process). */
struct ReplayPool {
    std::mutex call, m;
    std::condition_variable go, done;
    std::vector<std::thread> th;
    std::function<void(unsigned)> job;
    unsigned njob = 0, pending = 0;
    uint64_t gen = 0;

    pid_t owner = getpid();

    void run(unsigned T, const std::function<void(unsigned)> &fn) {
        std::lock_guard<std::mutex> serial(call);
        {
            std::unique_lock<std::mutex> lk(m);
            if (getpid() != owner) {
                /* a forked child inherits the pool but not its threads */
                th.clear();
                owner = getpid();
            }
            while (th.size() + 1 < T) {
                const unsigned id = (unsigned)th.size() + 1;
                th.emplace_back([this, id] { loop(id); });
                th.back().detach();
            }
            job = fn;
            njob = T;
            pending = T - 1;
            gen++;
        }
        go.notify_all();
        fn(0);
        std::unique_lock<std::mutex> lk(m);
        done.wait(lk, [&] { return pending == 0; });
        job = nullptr;
    }
    void loop(unsigned id) {
        uint64_t seen = 0;
        for (;;) {
            std::function<void(unsigned)> f;
            {
                std::unique_lock<std::mutex> lk(m);
                go.wait(lk, [&] { return gen != seen; });
                seen = gen;
                if (id >= njob) continue;
                f = job;
            }
            f(id);
            std::lock_guard<std::mutex> lk(m);
            if (--pending == 0) done.notify_one();
        }
    }
};
ReplayPool &replay_pool() {
    static ReplayPool *p = new ReplayPool();
    return *p;
}

vsa_db_t *device_db(vsa_hs_scratch_t *s, const vsa_hs_database_t *db) {
    for (auto &e : s->dbs)
        if (e.first == db->serial) return e.second;
    return nullptr;
}

/* one call's view of the stream: the writes of this call after the
 * history, and the match callback state */
struct Run {
    const vsa_hs_database *db;
    vsa_hs_stream *st;
    vsa_hs_match_event_handler cb;
    void *ctx;
    const uint8_t *const *bufs;
    const size_t *lens;
    std::vector<uint64_t> pos; /* stream offset of each write */
    size_t cur = 0;
    uint64_t last_to = ~0ULL;
    std::vector<uint32_t> at_to; /* ids reported at last_to */
    std::map<uint32_t, uint64_t> som_log; /* id -> leftmost from at last_to */
    bool terminated = false;
    std::vector<uint32_t> *touched = nullptr; /* corpus replay: ekeys set, to reset */
};

/* flushStoredSomMatches (src/som/som_runtime.c, report.h): the SOM reports
 * of deduped ids held for the current offset, leftmost start per id, in
 * dedupe-key (id) order */
bool flush_som(Run &r) {
    bool ok = true;
    for (const auto &e : r.som_log) {
        if (ok && r.cb && r.cb(e.first, e.second, r.last_to, 0, r.ctx)) {
            r.terminated = true;
            ok = false;
        }
    }
    r.som_log.clear();
    return ok;
}

uint8_t byte_at(const Run &r, uint64_t p) {
    if (p < r.pos[0]) return r.st->hist[r.st->hist.size() - (size_t)(r.pos[0] - p)];
    size_t j = r.cur;
    while (p < r.pos[j]) j--; /* earlier writes of this call */
    return r.bufs[j][p - r.pos[j]];
}

/* CHECK_LONG_LIT: the bytes of the literal before its matched 8-byte tail */
bool long_ok(const Run &r, uint64_t to, const Pattern &p) {
    const size_t len = p.s.size();
    if (to < len || to - len + r.st->hist.size() < r.st->offset) return false;
    const uint64_t start = to - len;
    for (size_t k = 0; k + SHORT_LIT < len; k++) {
        uint8_t b = byte_at(r, start + k);
        if (p.caseless) b = upper(b);
        if (b != (uint8_t)p.s[k]) return false;
    }
    return true;
}

u64a on_fragment(size_t end, u32 frag, hs_scratch *sc) {
    Run &r = *(Run *)sc;
    const uint64_t to = r.pos[r.cur] + end + 1; /* lit_offset_adjust */
    if (to != r.last_to) {
        if (!r.som_log.empty() && !flush_som(r)) return HWLM_TERMINATE_MATCHING;
        r.last_to = to;
        r.at_to.clear();
    }
    for (uint32_t pi : r.db->frags[frag]) {
        const Pattern &p = r.db->pats[pi];
        if (p.s.size() > SHORT_LIT && !long_ok(r, to, p)) continue;
        if (p.ekey != NO_EKEY && r.st->exhausted[p.ekey]) continue;
        if (p.som_dedupe) {
            const uint64_t from = to - p.s.size();
            auto it = r.som_log.find(p.id);
            if (it == r.som_log.end()) r.som_log.emplace(p.id, from);
            else it->second = std::min(it->second, from);
            continue;
        }
        if (r.db->dedupe) {
            if (std::find(r.at_to.begin(), r.at_to.end(), p.id) != r.at_to.end()) continue;
            r.at_to.push_back(p.id);
        }
        if (p.ekey != NO_EKEY) {
            r.st->exhausted[p.ekey] = 1;
            if (r.touched) r.touched->push_back(p.ekey);
        }
        const uint64_t from = p.som ? to - p.s.size() : 0;
        if (r.cb && r.cb(p.id, from, to, 0, r.ctx)) {
            r.terminated = true;
            return HWLM_TERMINATE_MATCHING;
        }
    }
    return HWLM_CONTINUE_MATCHING;
}

void on_piece(void *p, size_t i) { ((Run *)p)->cur = i; }

int count_match(unsigned, unsigned long long, unsigned long long, unsigned, void *ctx) {
    ++*(uint64_t *)ctx;
    return 0;
}

/* count + order-dependent digest of the callback sequence (vsa_hs_corpus_scan_ex) */
struct SeqDigest {
    uint64_t cnt = 0, h = 0;
};
int digest_match(unsigned id, unsigned long long from, unsigned long long to, unsigned,
                 void *ctx) {
    SeqDigest &d = *(SeqDigest *)ctx;
    d.cnt++;
    d.h = vsa_hs_seq_digest_step(d.h, id, from, to);
    return 0;
}

/* keep the last max(16, longest literal - 1) bytes of the stream */
void push_history(vsa_hs_stream *st, const uint8_t *const *bufs, const size_t *lens, size_t n) {
    const size_t keep = std::max(HIST_MIN, st->db->max_len ? st->db->max_len - 1 : 0);
    for (size_t i = 0; i < n; i++) {
        const size_t l = lens[i];
        if (!l) continue;
        if (l >= keep) {
            st->hist.assign(bufs[i] + l - keep, bufs[i] + l);
        } else {
            st->hist.insert(st->hist.end(), bufs[i], bufs[i] + l);
            if (st->hist.size() > keep)
                st->hist.erase(st->hist.begin(), st->hist.end() - keep);
        }
    }
}

/* the writes bufs[0, n) of one stream, in one GPU launch */
int scan_writes(vsa_hs_stream *st, vsa_hs_scratch_t *s, const uint8_t *const *bufs,
                const size_t *lens, size_t n, vsa_hs_match_event_handler cb, void *ctx) {
    vsa_db_t *ddb = device_db(s, st->db);
    if (!ddb) return VSA_HS_INVALID;
    Run r{st->db, st, cb, ctx, bufs, lens, {}, 0};
    r.pos.resize(n);
    uint64_t o = st->offset;
    for (size_t i = 0; i < n; i++) {
        r.pos[i] = o;
        o += lens[i];
    }
    const int rc = vsa::exec_pieces(s->ctx, ddb, st->hist.data(), st->hist.size(), bufs, lens,
                                    n, on_fragment, &r, on_piece);
    if (rc == HWLM_SUCCESS && !r.terminated) flush_som(r); /* end of the write */
    push_history(st, bufs, lens, n);
    st->offset = o;
    if (r.terminated) {
        st->terminated = true;
        return VSA_HS_SCAN_TERMINATED;
    }
    return rc == HWLM_SUCCESS ? VSA_HS_SUCCESS : VSA_HS_UNKNOWN_ERROR;
}

void init_stream(vsa_hs_stream *st, const vsa_hs_database *db) {
    st->db = db;
    st->offset = 0;
    st->hist.clear();
    st->exhausted.assign(db->n_ekeys, 0);
    st->terminated = false;
}

/* common entry checks: scratch valid for db, then marked in use */
int enter(const vsa_hs_database_t *db, vsa_hs_scratch_t *s) {
    if (!s || s->magic != SCRATCH_MAGIC || !device_db(s, db)) return VSA_HS_INVALID;
    if (s->in_use.exchange(true)) return VSA_HS_SCRATCH_IN_USE;
    return VSA_HS_SUCCESS;
}

void leave(vsa_hs_scratch_t *s) { s->in_use.store(false); }

} // namespace

extern "C" {

int vsa_hs_compile_lit_multi(const char *const *expressions, const unsigned *flags,
                             const unsigned *ids, const size_t *lens, unsigned elements,
                             unsigned mode, const void *platform, vsa_hs_database_t **db,
                             vsa_hs_compile_error_t **error) {
    (void)platform;
    /* hs.cpp:296-352 */
    if (!error) {
        if (db) *db = nullptr;
        return VSA_HS_COMPILER_ERROR;
    }
    auto fail = [&](const std::string &m, int idx) {
        if (db) *db = nullptr;
        *error = make_error(m, idx);
        return VSA_HS_COMPILER_ERROR;
    };
    if (!db) return fail("Invalid parameter: db is NULL", -1);
    if (!expressions) return fail("Invalid parameter: expressions is NULL", -1);
    if (!lens) return fail("Invalid parameter: len is NULL", -1);
    if (elements == 0) return fail("Invalid parameter: elements is zero", -1);
    const unsigned horizons = VSA_HS_MODE_SOM_HORIZON_LARGE | VSA_HS_MODE_SOM_HORIZON_MEDIUM |
                              VSA_HS_MODE_SOM_HORIZON_SMALL;
    const unsigned kinds = VSA_HS_MODE_BLOCK | VSA_HS_MODE_STREAM | VSA_HS_MODE_VECTORED;
    if (mode & ~(kinds | horizons))
        return fail("Invalid parameter: unrecognised mode flags.", -1);
    const unsigned kind = mode & kinds;
    if (!kind || (kind & (kind - 1)))
        return fail("Invalid parameter: mode must have one (and only one) of HS_MODE_BLOCK, "
                    "HS_MODE_STREAM or HS_MODE_VECTORED set.", -1);
    const unsigned som_mode = mode & horizons;
    if (som_mode) {
        if (!(mode & VSA_HS_MODE_STREAM))
            return fail("Invalid parameter: the HS_MODE_SOM_HORIZON_ mode flags may only be "
                        "set in streaming mode.", -1);
        if (som_mode & (som_mode - 1))
            return fail("Invalid parameter: only one HS_MODE_SOM_HORIZON_ mode flag can be "
                        "set.", -1);
    }
    if (elements > LIMIT_PATTERN_COUNT) return fail("Number of patterns too large", -1);

    vsa_hs_database *out = new (std::nothrow) vsa_hs_database;
    if (!out) return fail("Unable to allocate memory.", -1);
    out->mode = kind;
    out->mode_full = mode;
    out->serial = g_serial.fetch_add(1);
    std::map<uint32_t, std::pair<bool, unsigned>> ext; /* id -> (single, first index) */
    std::map<uint32_t, uint32_t> ekeys;
    std::map<uint32_t, uint32_t> ext_count; /* patterns per id */
    std::map<std::pair<std::string, bool>, uint32_t> frag_of;
    std::vector<vsa::Literal> lits;
    std::vector<bool> frag_noruns;
    const unsigned allowed = VSA_HS_FLAG_CASELESS | VSA_HS_FLAG_SINGLEMATCH |
                             VSA_HS_FLAG_SOM_LEFTMOST;
    const unsigned all_flags = 0x7ffu; /* HS_FLAG_ALL, hs_internal.h:75-85 */
    size_t min_len = ~(size_t)0;
    for (unsigned i = 0; i < elements; i++) {
        const unsigned f = flags ? flags[i] : 0;
        const uint32_t id = ids ? ids[i] : 0;
        const char *e = expressions[i];
        const int idx = (int)i;
        if (!e) {
            delete out;
            return fail("Invalid parameter: expression is NULL", idx);
        }
        /* compiler.cpp:406-423 */
        if (lens[i] > LIMIT_PATTERN_LENGTH) {
            delete out;
            return fail("Pattern length exceeds limit.", idx);
        }
        if (f & ~allowed & all_flags) {
            delete out;
            return fail("Only HS_FLAG_CASELESS, HS_FLAG_SINGLEMATCH and HS_FLAG_SOM_LEFTMOST "
                        "are supported in literal API.", idx);
        }
        if (e[0] == '\0' || lens[i] == 0) {
            delete out;
            return fail("Pure literal API doesn't support empty string.", idx);
        }
        /* compiler.cpp:130-139 */
        if (f & ~all_flags) {
            delete out;
            return fail("Unrecognised flag.", idx);
        }
        const bool single = f & VSA_HS_FLAG_SINGLEMATCH;
        if (single && (f & VSA_HS_FLAG_SOM_LEFTMOST)) {
            delete out;
            return fail("HS_FLAG_SINGLEMATCH is not supported in combination with "
                        "HS_FLAG_SOM_LEFTMOST.", idx);
        }
        /* report_manager.cpp:212-236 */
        auto it = ext.find(id);
        if (it == ext.end()) {
            ext.emplace(id, std::make_pair(single, i));
        } else {
            out->dedupe = true;
            if (it->second.first != single) {
                std::string m = "Expression (index " + std::to_string(i) + ") with match ID " +
                                std::to_string(id) + " " +
                                (single ? "specified " : "did not specify ") +
                                "HS_FLAG_SINGLEMATCH whereas previous expression (index " +
                                std::to_string(it->second.second) +
                                ") with the same match ID did" + (single ? " not" : "") + ".";
                delete out;
                return fail(m, idx);
            }
        }
        ext_count[id]++;
        out->src.push_back({std::string(e, lens[i]), f, id});
        Pattern p;
        p.id = id;
        p.som = f & VSA_HS_FLAG_SOM_LEFTMOST;
        p.caseless = f & VSA_HS_FLAG_CASELESS;
        p.s.assign(e, lens[i]);
        if (p.caseless)
            for (auto &c : p.s) c = (char)upper((uint8_t)c);
        if (single) {
            auto ek = ekeys.find(id);
            if (ek == ekeys.end()) ek = ekeys.emplace(id, (uint32_t)ekeys.size()).first;
            p.ekey = ek->second;
        }
        const std::string tail = p.s.size() > SHORT_LIT ? p.s.substr(p.s.size() - SHORT_LIT) : p.s;
        const auto key = std::make_pair(tail, p.caseless);
        auto fr = frag_of.find(key);
        if (fr == frag_of.end()) {
            fr = frag_of.emplace(key, (uint32_t)out->frags.size()).first;
            out->frags.emplace_back();
            frag_noruns.push_back(true);
            lits.push_back(vsa::makeLiteral((const u8 *)tail.data(), tail.size(), p.caseless,
                                            false, fr->second, HWLM_ALL_GROUPS, nullptr,
                                            nullptr, 0));
        }
        if (!single || p.s.size() > SHORT_LIT) frag_noruns[fr->second] = false;
        out->frags[fr->second].push_back((uint32_t)out->pats.size());
        out->max_len = std::max(out->max_len, p.s.size());
        min_len = std::min(min_len, p.s.size());
        out->pats.push_back(std::move(p));
    }
    for (size_t k = 0; k < lits.size(); k++) lits[k].noruns = frag_noruns[k];
    for (auto &p : out->pats)
        if (p.som && ext.count(p.id) && ext_count[p.id] > 1) p.som_dedupe = true;
    out->n_ekeys = (uint32_t)ekeys.size();
    out->simple = !out->dedupe && out->n_ekeys == 0 && out->max_len <= SHORT_LIT &&
                  std::all_of(out->frags.begin(), out->frags.end(),
                              [](const std::vector<uint32_t> &f) { return f.size() == 1; });
    out->min_width = (uint32_t)min_len;
    vsa::BuildOptions opt;
    if (vsa::buildHwlm(lits, opt, &out->hwlm, &out->hwlm_size) != VSA_OK) {
        delete out;
        return fail("Internal error.", -1);
    }
    *db = out;
    *error = nullptr;
    return VSA_HS_SUCCESS;
}

int vsa_hs_compile_lit(const char *expression, unsigned flags, size_t len, unsigned mode,
                       const void *platform, vsa_hs_database_t **db,
                       vsa_hs_compile_error_t **error) {
    const unsigned id = 0;
    return vsa_hs_compile_lit_multi(&expression, &flags, &id, &len, 1, mode, platform, db,
                                    error);
}

int vsa_hs_free_compile_error(vsa_hs_compile_error_t *error) {
    if (error) {
        free(error->message);
        free(error);
    }
    return VSA_HS_SUCCESS;
}

int vsa_hs_free_database(vsa_hs_database_t *db) {
    if (db && db->magic != DB_MAGIC) return VSA_HS_INVALID;
    if (db) {
        db->magic = 0;
        vsa_blob_free(db->hwlm);
        delete db;
    }
    return VSA_HS_SUCCESS;
}

int vsa_hs_database_hwlm(const vsa_hs_database_t *db, const void **hwlm, size_t *size,
                         unsigned *fragments) {
    if (!valid_db(db)) return VSA_HS_INVALID;
    if (hwlm) *hwlm = db->hwlm;
    if (size) *size = db->hwlm_size;
    if (fragments) *fragments = (unsigned)db->frags.size();
    return VSA_HS_SUCCESS;
}

/* scratch.c:242-300: grows an existing scratch to serve db as well */
int vsa_hs_alloc_scratch(const vsa_hs_database_t *db, vsa_hs_scratch_t **scratch) {
    if (!db || !scratch) return VSA_HS_INVALID;
    if (!valid_db(db)) return VSA_HS_INVALID;
    vsa_hs_scratch_t *s = *scratch;
    if (s) {
        if (s->magic != SCRATCH_MAGIC) return VSA_HS_INVALID;
        if (s->in_use.exchange(true)) return VSA_HS_SCRATCH_IN_USE;
    } else {
        s = new (std::nothrow) vsa_hs_scratch;
        if (!s) return VSA_HS_NOMEM;
        s->in_use.store(true);
        const char *e = getenv("VSA_DEVICE");
        if (vsa_ctx_create(e ? atoi(e) : 0, &s->ctx) != VSA_OK) {
            delete s;
            return VSA_HS_NOMEM;
        }
    }
    if (!device_db(s, db)) {
        vsa_db_t *d = nullptr;
        if (vsa_db_load(s->ctx, db->hwlm, db->hwlm_size, &d) != VSA_OK) {
            s->in_use.store(false);
            if (!*scratch) vsa_hs_free_scratch(s);
            return VSA_HS_NOMEM;
        }
        s->dbs.emplace_back(db->serial, d);
    }
    s->in_use.store(false);
    *scratch = s;
    return VSA_HS_SUCCESS;
}

int vsa_hs_free_scratch(vsa_hs_scratch_t *scratch) {
    if (!scratch) return VSA_HS_SUCCESS;
    if (scratch->magic != SCRATCH_MAGIC) return VSA_HS_INVALID;
    if (scratch->in_use.exchange(true)) return VSA_HS_SCRATCH_IN_USE;
    for (auto &e : scratch->dbs) vsa_db_free(e.second);
    if (scratch->ctx) vsa_ctx_destroy(scratch->ctx);
    scratch->magic = 0;
    delete scratch;
    return VSA_HS_SUCCESS;
}

/* runtime.c:316-470 */
int vsa_hs_scan(const vsa_hs_database_t *db, const char *data, unsigned int length,
                unsigned int flags, vsa_hs_scratch_t *scratch,
                vsa_hs_match_event_handler onEvent, void *context) {
    (void)flags;
    if (!scratch || !data) return VSA_HS_INVALID;
    if (!valid_db(db)) return VSA_HS_INVALID;
    if (db->mode != VSA_HS_MODE_BLOCK) return VSA_HS_DB_MODE_ERROR;
    int rc = enter(db, scratch);
    if (rc != VSA_HS_SUCCESS) return rc;
    if (db->min_width > length) {
        leave(scratch);
        return VSA_HS_SUCCESS;
    }
    vsa_hs_stream st;
    init_stream(&st, db);
    const uint8_t *b = (const uint8_t *)data;
    const size_t l = length;
    rc = scan_writes(&st, scratch, &b, &l, 1, onEvent, context);
    leave(scratch);
    return rc;
}

/* runtime.c:1106-1180: pieces up to the first NULL one are scanned (its
 * hs_scan_stream_internal call fails with HS_INVALID) */
int vsa_hs_scan_vector(const vsa_hs_database_t *db, const char *const *data,
                       const unsigned int *length, unsigned int count, unsigned int flags,
                       vsa_hs_scratch_t *scratch, vsa_hs_match_event_handler onEvent,
                       void *context) {
    (void)flags;
    if (!scratch || !data || !length) return VSA_HS_INVALID;
    if (!valid_db(db)) return VSA_HS_INVALID;
    if (db->mode != VSA_HS_MODE_VECTORED) return VSA_HS_DB_MODE_ERROR;
    int rc = enter(db, scratch);
    if (rc != VSA_HS_SUCCESS) return rc;
    unsigned n = 0;
    while (n < count && data[n]) n++;
    std::vector<size_t> lens(length, length + n);
    vsa_hs_stream st;
    init_stream(&st, db);
    /* one launch holds at most VSA_MAX_BLOCKS non-empty pieces (empty ones
     * are not launched): a longer vector is scanned as consecutive launches
     * of the same stream, its state (offset, history, exhaustion) carried
     * across, which is what the reference's per-piece stream writes do */
    const uint8_t *const *bufs = (const uint8_t *const *)data;
    for (unsigned i0 = 0; i0 < n && rc == VSA_HS_SUCCESS;) {
        unsigned i1 = i0, live = 0;
        while (i1 < n && (live < VSA_MAX_BLOCKS || !lens[i1])) live += lens[i1++] != 0;
        rc = scan_writes(&st, scratch, bufs + i0, lens.data() + i0, i1 - i0, onEvent, context);
        i0 = i1;
    }
    leave(scratch);
    if (rc != VSA_HS_SUCCESS) return rc;
    return n < count ? VSA_HS_INVALID : VSA_HS_SUCCESS;
}

/* The corpus loop of hsbench (tools/hsbench/main.cpp:487-511 block mode,
 * :520-600 streaming / vectored) as ONE launch over device-resident blocks.
 * Block database: every block is one hs_scan.  Stream / vectored database:
 * the blocks of one stream_ids value, in array order, are the writes of one
 * stream and must lie back to back in d_data (each block's history is what
 * precedes it).  counts[b] (optional) = matches of block b after the report
 * program; *total = their sum.  h_data = host copy of d_data's bytes (needed
 * only for literals longer than 8 bytes).  A database where every HWLM
 * record is exactly one report (distinct ids, literals <= 8 bytes, no
 * SINGLEMATCH) takes *total from the GPU's record count without copying the
 * records back; otherwise the records are replayed through the report
 * program on `threads` host threads (streams are independent).  No match
 * callbacks: this is the benchmark path.  A prepared corpus keeps the
 * launch plan (block table, segment map) and the stream grouping on the
 * device / host between scans. */
struct vsa_hs_corpus {
    const vsa_hs_database *db = nullptr;
    vsa_hs_scratch *scratch = nullptr;
    const uint8_t *d_data = nullptr, *h_data = nullptr;
    std::vector<uint64_t> offsets, lens;
    bool streams = false;
    /* units = streams (or single blocks), CSR: unit u is blocks
     * unit_blk[unit_off[u] .. unit_off[u + 1]) in write order */
    std::vector<uint32_t> unit_off, unit_blk, blk_unit;
    std::vector<uint32_t> order;  /* non-empty blocks by offset */
    std::vector<uint64_t> so, se; /* their [offset, end) in that order */
    /* per-scan record ranges, valid where bstamp == gen (no clearing) */
    std::vector<uint64_t> rb, re;
    std::vector<uint32_t> bstamp, ustamp;
    uint32_t gen = 0;
    vsa_plan_t *plan = nullptr;
    /* block mode, every block the same length L (the last may be shorter)
     * and laid back to back from off0 (hsbench's fixed-size chunks): the
     * block of an end is (end - off0) / L, no search */
    bool uniform = false;
    uint64_t off0 = 0, ulen = 0;
    std::vector<uint32_t> empty; /* zero-length blocks (not in `order`) */
    /* the plan's inputs (non-empty blocks), and the second context (on the
     * scratch context's stream) with its own plan of them that the
     * pipelined repeat loop alternates with: made at its first use */
    std::vector<uint64_t> p_off, p_len, p_hist;
    vsa_ctx_t *ctx2 = nullptr;
    vsa_plan_t *plan2 = nullptr;
};

int vsa_hs_corpus_prepare(const vsa_hs_database_t *db, vsa_hs_scratch_t *scratch,
                          const uint8_t *d_data, const uint8_t *h_data,
                          const uint64_t *offsets, const uint64_t *lens,
                          const uint32_t *stream_ids, uint32_t nblocks,
                          vsa_hs_corpus_t **out) {
    if (!valid_db(db) || !offsets || !lens || !out || (nblocks && !d_data))
        return VSA_HS_INVALID;
    /* one launch plan per corpus: at most VSA_MAX_BLOCKS chunks (the
     * reference has no such limit; a larger corpus is prepared in parts) */
    if (nblocks > VSA_MAX_BLOCKS) return VSA_HS_INVALID;
    if (db->max_len > SHORT_LIT && !h_data) return VSA_HS_INVALID;
    if (!scratch || scratch->magic != SCRATCH_MAGIC || !device_db(scratch, db))
        return VSA_HS_INVALID;
    vsa_hs_corpus *c = new (std::nothrow) vsa_hs_corpus;
    if (!c) return VSA_HS_NOMEM;
    c->db = db;
    c->scratch = scratch;
    c->d_data = d_data;
    c->h_data = h_data;
    c->offsets.assign(offsets, offsets + nblocks);
    c->lens.assign(lens, lens + nblocks);
    c->streams = db->mode != VSA_HS_MODE_BLOCK && stream_ids;
    std::map<uint32_t, std::vector<uint32_t>> by_stream;
    std::vector<uint64_t> hl(nblocks, 0);
    std::vector<uint64_t> lo, ln, lh;
    for (uint32_t b = 0; b < nblocks; b++) {
        if (c->streams) {
            auto &v = by_stream[stream_ids[b]];
            if (!v.empty()) {
                const uint32_t p = v.back();
                if (offsets[b] != offsets[p] + lens[p]) {
                    delete c;
                    return VSA_HS_INVALID;
                }
                hl[b] = std::min<uint64_t>(16, hl[p] + lens[p]);
            }
            v.push_back(b);
        }
        if (lens[b]) {
            c->order.push_back(b);
            lo.push_back(offsets[b]);
            ln.push_back(lens[b]);
            lh.push_back(hl[b]);
        }
    }
    c->blk_unit.assign(nblocks, 0);
    c->unit_off.push_back(0);
    if (c->streams) {
        for (auto &e : by_stream) {
            for (uint32_t b : e.second) {
                c->blk_unit[b] = (uint32_t)c->unit_off.size() - 1;
                c->unit_blk.push_back(b);
            }
            c->unit_off.push_back((uint32_t)c->unit_blk.size());
        }
    } else {
        for (uint32_t b = 0; b < nblocks; b++) {
            c->blk_unit[b] = b;
            c->unit_blk.push_back(b);
            c->unit_off.push_back(b + 1);
        }
    }
    std::stable_sort(c->order.begin(), c->order.end(),
                     [&](uint32_t a, uint32_t b) { return offsets[a] < offsets[b]; });
    for (uint32_t b : c->order) {
        c->so.push_back(offsets[b]);
        c->se.push_back(offsets[b] + lens[b]);
    }
    if (!c->streams) {
        for (uint32_t b = 0; b < nblocks; b++)
            if (!lens[b]) c->empty.push_back(b);
        c->uniform = nblocks > 0 && c->empty.empty() && lens[0] > 0;
        for (uint32_t b = 0; c->uniform && b < nblocks; b++)
            c->uniform = offsets[b] == offsets[0] + (uint64_t)b * lens[0] &&
                         (lens[b] == lens[0] || (b + 1 == nblocks && lens[b] < lens[0]));
        c->off0 = nblocks ? offsets[0] : 0;
        c->ulen = nblocks ? lens[0] : 0;
    }
    c->rb.assign(nblocks, 0);
    c->re.assign(nblocks, 0);
    c->bstamp.assign(nblocks, 0);
    c->ustamp.assign(c->unit_off.size() - 1, 0);
    if (!lo.empty() &&
        vsa_plan_create(scratch->ctx, d_data, lo.data(), ln.data(), nullptr,
                        c->streams ? lh.data() : nullptr, nullptr, (uint32_t)lo.size(),
                        &c->plan) != VSA_OK) {
        delete c;
        return VSA_HS_NOMEM;
    }
    c->p_off = std::move(lo);
    c->p_len = std::move(ln);
    c->p_hist = std::move(lh);
    *out = c;
    return VSA_HS_SUCCESS;
}

int vsa_hs_corpus_free(vsa_hs_corpus_t *c) {
    if (!c) return VSA_HS_SUCCESS;
    vsa_plan_free(c->plan);
    vsa_plan_free(c->plan2);
    if (c->ctx2) vsa_ctx_destroy(c->ctx2);
    delete c;
    return VSA_HS_SUCCESS;
}

/* Block mode (a unit is one block): the records, sorted by end, are cut
 * into T contiguous ranges at block boundaries and each thread maps AND
 * replays its own range -- no serial record-to-block pass, and each thread
 * zeroes the counts / digests of the blocks between its first and the next
 * thread's first (positions in `order`), so blocks without records cost one
 * store each, in parallel.  Same results as the unit path: every block is
 * an independent hs_scan. */
static int corpus_replay_blocks(vsa_hs_corpus *cp, uint64_t *keys, const uint32_t *ids,
                                uint64_t nm, uint64_t *counts, uint64_t *digests,
                                uint64_t *total, unsigned threads) {
    const auto t_start = std::chrono::steady_clock::now();
    const vsa_hs_database *db = cp->db;
    vsa_db_t *ddb = device_db(cp->scratch, db);
    const uint64_t *lens = cp->lens.data();
    const auto &so = cp->so, &se = cp->se;
    const size_t npos = so.size();
    *total = 0;
    for (uint32_t b : cp->empty) {
        if (counts) counts[b] = 0;
        if (digests) digests[b] = 0;
    }
    /* the position in `order` of the block holding end e, searching
     * forward from `at` (the previous record's position); npos = none */
    auto pos_of = [&](uint64_t e, size_t at) -> size_t {
        if (cp->uniform) {
            if (e < cp->off0) return npos;
            const uint64_t p = (e - cp->off0) / cp->ulen;
            return p < npos && e < se[p] ? (size_t)p : npos;
        }
        size_t lo = at, step = 1;
        while (lo + step < npos && so[lo + step] <= e) {
            lo += step;
            step <<= 1;
        }
        const size_t oi = (size_t)(std::upper_bound(so.begin() + lo,
                                                    so.begin() + std::min(npos, lo + step), e) -
                                   so.begin());
        return oi && e < se[oi - 1] ? oi - 1 : npos;
    };
    /* a thread per ~2k records (thread start-up costs more than replaying a
     * few hundred) */
    const unsigned T = (unsigned)std::max<uint64_t>(
        1, std::min<uint64_t>({threads ? threads : 1u, 1 + nm / 2048, npos ? npos : 1}));
    /* range t = records [kt[t], kt[t + 1]), block positions [pt[t], pt[t + 1]) */
    std::vector<uint64_t> kt(T + 1, nm);
    std::vector<size_t> pt(T + 1, npos);
    kt[0] = 0;
    pt[0] = 0;
    for (unsigned t = 1; t < T; t++) {
        uint64_t k = std::max(kt[t - 1], nm * t / T);
        size_t p = npos;
        for (; k < nm; k++) {
            const uint64_t e = keys[k] >> KEY_END_SHIFT;
            const size_t lo = (size_t)(std::upper_bound(so.begin(), so.end(), e) - so.begin());
            p = lo && e < se[lo - 1] ? lo - 1 : npos;
            if (p != npos) break;
        }
        if (p == npos || p < pt[t - 1]) { /* the rest belongs to range t - 1 */
            for (unsigned u = t; u < T; u++) {
                kt[u] = nm;
                pt[u] = npos;
            }
            break;
        }
        /* to the nearer block boundary: back to the block's first record,
         * or on to the next block's (few large blocks: snapping back alone
         * left one thread two blocks and another none) */
        const uint64_t k_lo = (uint64_t)(std::lower_bound(keys + kt[t - 1], keys + k,
                                                          (uint64_t)so[p] << KEY_END_SHIFT) - keys);
        const uint64_t k_hi =
            p + 1 < npos ? (uint64_t)(std::lower_bound(keys + k, keys + nm,
                                                       (uint64_t)so[p + 1] << KEY_END_SHIFT) -
                                      keys)
                         : nm;
        if ((k_lo <= kt[t - 1] || k - k_lo > k_hi - k) && p + 1 < npos) {
            kt[t] = k_hi;
            pt[t] = p + 1;
        } else {
            kt[t] = k_lo;
            pt[t] = p;
        }
    }
    std::vector<uint64_t> part(T, 0);
    std::vector<int> status(T, VSA_HS_SUCCESS);
    std::vector<double> busy(T, 0.0);
    using clk = std::chrono::steady_clock;
    const auto t_split = clk::now();
    const uint8_t *h_data = cp->h_data;
    auto work = [&](unsigned t) {
        const auto w0 = clk::now();
        for (size_t p = pt[t]; p < pt[t + 1]; p++) {
            const uint32_t b = cp->order[p];
            if (counts) counts[b] = 0;
            if (digests) digests[b] = 0;
        }
        vsa_hs_stream st;
        init_stream(&st, db);
        std::vector<uint32_t> touched;
        const uint8_t *buf = nullptr;
        size_t blen = 0;
        SeqDigest dg;
        uint64_t &cnt = dg.cnt;
        Run r{db, &st, digests ? digest_match : count_match, digests ? (void *)&dg : (void *)&cnt,
              &buf, &blen, {0}, 0};
        r.touched = &touched;
        size_t at = pt[t];
        uint64_t k = kt[t];
        const uint64_t k_end = kt[t + 1];
        while (k < k_end) {
            const uint64_t e = keys[k] >> KEY_END_SHIFT;
            const size_t p = pos_of(e, at);
            if (p == npos) { /* outside every block: not reported */
                k++;
                continue;
            }
            at = p;
            const uint32_t b = cp->order[p];
            const uint64_t o = so[p], hi = se[p];
            const uint64_t k0 = k;
            while (k < k_end && (keys[k] >> KEY_END_SHIFT) < hi) {
                keys[k] -= o << KEY_END_SHIFT;
                k++;
            }
            /* a fresh hs_scan of block b: the previous block's exhaustion
             * keys reset, nothing else carried */
            for (uint32_t x : touched) st.exhausted[x] = 0;
            touched.clear();
            cnt = 0;
            dg.h = 0;
            buf = h_data ? h_data + o : nullptr;
            blen = lens[b];
            r.last_to = ~0ULL;
            r.at_to.clear();
            r.som_log.clear();
            r.terminated = false;
            if (vsa::replay_records(ddb, keys + k0, ids + k0, k - k0, on_fragment, &r) !=
                HWLM_SUCCESS) {
                status[t] = VSA_HS_UNKNOWN_ERROR;
                return;
            }
            flush_som(r);
            if (counts) counts[b] = cnt;
            if (digests) digests[b] = dg.h;
            part[t] += cnt;
        }
        busy[t] = std::chrono::duration<double, std::milli>(clk::now() - w0).count();
    };
    if (T == 1) work(0);
    else replay_pool().run(T, work);
    static const bool timing = getenv("VSA_HOST_TIMING") != nullptr;
    if (timing) {
        double mx = 0, sum = 0;
        for (double x : busy) {
            mx = std::max(mx, x);
            sum += x;
        }
        fprintf(stderr, "corpus_replay_blocks: %u threads, %llu records, %zu blocks: split %.3f ms, "
                "replay %.3f ms (thread busy max %.3f, mean %.3f ms)\n", T,
                (unsigned long long)nm, npos,
                std::chrono::duration<double, std::milli>(t_split - t_start).count(),
                std::chrono::duration<double, std::milli>(clk::now() - t_split).count(), mx,
                sum / T);
    }
    for (unsigned t = 0; t < T; t++) {
        if (status[t] != VSA_HS_SUCCESS) return status[t];
        *total += part[t];
    }
    return VSA_HS_SUCCESS;
}

/* The records of one corpus scan (sorted by d_data end offset; keys are
 * rebased to their block in place) through the report program on
 * `threads` host threads: per-block counts / sequence digests (optional)
 * and the total. */
static int corpus_replay(vsa_hs_corpus *cp, uint64_t *keys, const uint32_t *ids, uint64_t nm,
                         uint64_t *counts, uint64_t *digests, uint64_t *total,
                         unsigned threads) {
    if (!cp->streams && !getenv("VSA_REPLAY_UNITS"))
        return corpus_replay_blocks(cp, keys, ids, nm, counts, digests, total, threads);
    const auto t_start = std::chrono::steady_clock::now();
    const vsa_hs_database *db = cp->db;
    vsa_db_t *ddb = device_db(cp->scratch, db);
    const uint32_t nblocks = (uint32_t)cp->offsets.size();
    const uint64_t *offsets = cp->offsets.data(), *lens = cp->lens.data();
    if (counts) std::fill(counts, counts + nblocks, 0);
    if (digests) std::fill(digests, digests + nblocks, 0);
    *total = 0;
    /* records -> blocks: the records are sorted by end (d_data offsets),
     * the non-empty blocks by offset; each run of records is placed with one
     * binary search, so the cost follows the records, not the block count.
     * Units holding records are the live ones (the others report nothing,
     * their counts stay 0). */
    if (++cp->gen == 0) {
        std::fill(cp->bstamp.begin(), cp->bstamp.end(), 0);
        std::fill(cp->ustamp.begin(), cp->ustamp.end(), 0);
        cp->gen = 1;
    }
    const uint32_t gen = cp->gen;
    uint64_t *rb = cp->rb.data(), *re = cp->re.data();
    const uint32_t *bstamp = cp->bstamp.data();
    std::vector<uint32_t> live;
    uint64_t live_recs = 0;
    const auto &so = cp->so, &se = cp->se;
    /* the records of [k, k_end) -> blocks (each run with one gallop from the
     * previous run's block plus a binary search); their units, in order,
     * consecutive repeats dropped */
    auto map_range = [&](uint64_t k, uint64_t k_end, std::vector<uint32_t> &units,
                         uint64_t &recs) {
        size_t at = (size_t)(std::upper_bound(so.begin(), so.end(),
                                              k < k_end ? keys[k] >> KEY_END_SHIFT : 0) -
                             so.begin());
        at = at ? at - 1 : 0;
        uint32_t last_u = ~0u;
        while (k < k_end) {
            const uint64_t e = keys[k] >> KEY_END_SHIFT;
            size_t lo = at, step = 1;
            while (lo + step < so.size() && so[lo + step] <= e) {
                lo += step;
                step <<= 1;
            }
            const size_t oi = (size_t)(std::upper_bound(so.begin() + lo,
                                                        so.begin() + std::min(so.size(), lo + step),
                                                        e) - so.begin());
            at = oi ? oi - 1 : 0;
            if (oi == 0 || e >= se[oi - 1]) { /* outside every block: not reported */
                k++;
                continue;
            }
            const uint32_t b = cp->order[oi - 1];
            const uint64_t o = so[oi - 1], hi = se[oi - 1];
            const uint64_t k0 = k;
            while (k < k_end && (keys[k] >> KEY_END_SHIFT) < hi) {
                keys[k] -= o << KEY_END_SHIFT;
                k++;
            }
            rb[b] = k0;
            re[b] = k;
            cp->bstamp[b] = gen;
            const uint32_t u = cp->blk_unit[b];
            if (u != last_u) {
                units.push_back(u);
                last_u = u;
            }
            recs += k - k0;
        }
    };
    /* one thread: splitting the map over the replay pool measured slower
     * (pool hand-off and cache traffic outweigh ~10 ns per record) */
    {
        std::vector<uint32_t> units;
        map_range(0, nm, units, live_recs);
        for (uint32_t u : units) {
            if (cp->ustamp[u] != gen) {
                cp->ustamp[u] = gen;
                live.push_back(u);
            }
        }
    }
    const uint32_t *unit_off = cp->unit_off.data(), *unit_blk = cp->unit_blk.data();
    const uint8_t *h_data = cp->h_data;
    const bool streams = cp->streams;
    /* a thread per ~2k records (thread start-up costs more than replaying a
     * few hundred) */
    const unsigned T = (unsigned)std::max<uint64_t>(
        1, std::min<uint64_t>({threads ? threads : 1u, live.size(), 1 + live_recs / 2048}));
    std::vector<uint64_t> part(T, 0);
    std::vector<int> status(T, VSA_HS_SUCCESS);
    static const bool timing = getenv("VSA_HOST_TIMING") != nullptr;
    using clk = std::chrono::steady_clock;
    const auto t_map = clk::now();
    std::vector<double> busy(T, 0.0);
    auto work = [&](unsigned t) {
        const auto w0 = clk::now();
        /* per-thread state, reused across units: a unit resets only the
         * exhaustion keys the previous one set */
        vsa_hs_stream st;
        init_stream(&st, db);
        std::vector<uint32_t> touched;
        std::vector<const uint8_t *> bufs;
        std::vector<size_t> bl_len;
        SeqDigest dg;
        uint64_t &cnt = dg.cnt;
        Run r{db, &st, digests ? digest_match : count_match, digests ? (void *)&dg : (void *)&cnt,
              nullptr, nullptr, {}, 0};
        r.touched = &touched;
        /* contiguous slices of the live units (neighbouring blocks share
         * cache lines of the records, rb/re and the corpus image) */
        const size_t u0 = live.size() * t / T, u1 = live.size() * (t + 1) / T;
        for (size_t i = u0; i < u1; i++) {
            const uint32_t *bl = unit_blk + unit_off[live[i]];
            const size_t nbl = unit_off[live[i] + 1] - unit_off[live[i]];
            st.offset = 0;
            st.hist.clear();
            st.terminated = false;
            for (uint32_t k : touched) st.exhausted[k] = 0;
            touched.clear();
            cnt = 0;
            bufs.resize(nbl);
            bl_len.resize(nbl);
            for (size_t j = 0; j < nbl; j++) {
                bufs[j] = h_data ? h_data + offsets[bl[j]] : nullptr;
                bl_len[j] = lens[bl[j]];
            }
            r.bufs = bufs.data();
            r.lens = bl_len.data();
            r.cur = 0;
            r.last_to = ~0ULL;
            r.at_to.clear();
            r.som_log.clear();
            r.terminated = false;
            r.pos.resize(nbl);
            uint64_t o = 0;
            for (size_t j = 0; j < nbl; j++) {
                r.pos[j] = o;
                o += bl_len[j];
            }
            for (size_t j = 0; j < nbl; j++) {
                const uint32_t b = bl[j];
                const uint64_t before = cnt;
                dg.h = 0;
                r.cur = j;
                if (bstamp[b] == gen && re[b] > rb[b] &&
                    vsa::replay_records(ddb, keys + rb[b], ids + rb[b],
                                        re[b] - rb[b], on_fragment, &r) != HWLM_SUCCESS) {
                    status[t] = VSA_HS_UNKNOWN_ERROR;
                    return;
                }
                flush_som(r);
                if (streams && h_data) push_history(&st, &bufs[j], &bl_len[j], 1);
                st.offset += bl_len[j];
                if (counts) counts[b] = cnt - before;
                if (digests) digests[b] = dg.h;
            }
            part[t] += cnt;
        }
        busy[t] = std::chrono::duration<double, std::milli>(clk::now() - w0).count();
    };
    if (T == 1) work(0);
    else replay_pool().run(T, work);
    if (timing) {
        double mx = 0, sum = 0;
        for (double b : busy) {
            mx = std::max(mx, b);
            sum += b;
        }
        fprintf(stderr, "corpus_replay: %u threads, %zu live units, %llu records: map %.3f ms, "
                "replay %.3f ms (thread busy max %.3f, mean %.3f ms)\n", T, live.size(),
                (unsigned long long)live_recs,
                std::chrono::duration<double, std::milli>(t_map - t_start).count(),
                std::chrono::duration<double, std::milli>(clk::now() - t_map).count(), mx,
                sum / T);
    }
    for (unsigned t = 0; t < T; t++) {
        if (status[t] != VSA_HS_SUCCESS) return status[t];
        *total += part[t];
    }
    return VSA_HS_SUCCESS;
}


int vsa_hs_corpus_scan(vsa_hs_corpus_t *cp, uint64_t *counts, uint64_t *total,
                       unsigned threads) {
    return vsa_hs_corpus_scan_ex(cp, counts, nullptr, total, threads);
}

int vsa_hs_corpus_scan_ex(vsa_hs_corpus_t *cp, uint64_t *counts, uint64_t *digests,
                          uint64_t *total, unsigned threads) {
    if (!cp || !total || !valid_db(cp->db)) return VSA_HS_INVALID;
    const vsa_hs_database *db = cp->db;
    vsa_hs_scratch *scratch = cp->scratch;
    int rc = enter(db, scratch);
    if (rc != VSA_HS_SUCCESS) return rc;
    vsa_db_t *ddb = device_db(scratch, db);
    const uint32_t nblocks = (uint32_t)cp->offsets.size();
    if (counts) std::fill(counts, counts + nblocks, 0);
    if (digests) std::fill(digests, digests + nblocks, 0);
    *total = 0;
    const bool fast = db->simple && !counts && !digests;
    /* VSA_HOST_TIMING: per-phase wall times on stderr */
    static const bool timing = getenv("VSA_HOST_TIMING") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const auto t0 = now();
    std::vector<uint64_t> keys;
    std::vector<uint32_t> ids;
    uint64_t nm = 0;
    if (cp->plan &&
        vsa::scan_records(scratch->ctx, ddb, cp->d_data, nullptr, nullptr, nullptr, 0,
                          fast ? nullptr : &keys, fast ? nullptr : &ids, &nm,
                          cp->plan) != VSA_OK) {
        leave(scratch);
        return VSA_HS_UNKNOWN_ERROR;
    }
    if (fast) {
        *total = nm;
        leave(scratch);
        return VSA_HS_SUCCESS;
    }
    const auto t1 = now();
    rc = corpus_replay(cp, keys.data(), ids.data(), nm, counts, digests, total, threads);
    if (timing)
        fprintf(stderr, "vsa_hs_corpus_scan: scan+copy %.3f ms, map+replay %.3f ms (%llu records)\n",
                ms(t0, t1), ms(t1, now()), (unsigned long long)nm);
    leave(scratch);
    return rc;
}

/* hsbench's repeat loop (main.cpp:487-511, `repeats` passes over the
 * corpus) pipelined two passes deep over two contexts on one stream: while
 * the host replays pass k through the report program, passes k + 1 and
 * k + 2 are already queued on the GPU, so a pass costs max(scan + copy,
 * replay) and the GPU does not wait for the host between passes (one pass
 * ahead, as in round 5, left it idle for the host's turnaround: 1.0 against
 * 0.82 ms per 4 GiB pass end to end).  totals[k] = the matches of pass k;
 * counts / digests (optional) are those of the last pass.  Every pass scans
 * the whole corpus and replays all its records. */
int vsa_hs_corpus_scan_repeats(vsa_hs_corpus_t *cp, uint32_t repeats, uint64_t *totals,
                               uint64_t *counts, uint64_t *digests, unsigned threads) {
    if (!cp || !totals || !repeats || !valid_db(cp->db)) return VSA_HS_INVALID;
    const vsa_hs_database *db = cp->db;
    if (db->simple && !counts && !digests) {
        /* one record = one match: the GPU's counts, nothing to replay */
        for (uint32_t k = 0; k < repeats; k++) {
            int rc = vsa_hs_corpus_scan_ex(cp, nullptr, nullptr, &totals[k], threads);
            if (rc != VSA_HS_SUCCESS) return rc;
        }
        return VSA_HS_SUCCESS;
    }
    vsa_hs_scratch *scratch = cp->scratch;
    int rc = enter(db, scratch);
    if (rc != VSA_HS_SUCCESS) return rc;
    vsa_db_t *ddb = device_db(scratch, db);
    if (!cp->plan) {
        std::fill(totals, totals + repeats, 0);
        if (counts) std::fill(counts, counts + cp->offsets.size(), 0);
        if (digests) std::fill(digests, digests + cp->offsets.size(), 0);
        leave(scratch);
        return VSA_HS_SUCCESS;
    }
    /* two contexts on the scratch context's stream, each with its own plan,
     * results and counters: pass k runs on cx[k & 1] */
    if (repeats > 1 && !cp->ctx2) {
        if (vsa_ctx_create_shared(scratch->ctx, &cp->ctx2) != VSA_OK ||
            vsa_plan_create(cp->ctx2, cp->d_data, cp->p_off.data(), cp->p_len.data(), nullptr,
                            cp->streams ? cp->p_hist.data() : nullptr, nullptr,
                            (uint32_t)cp->p_off.size(), &cp->plan2) != VSA_OK) {
            if (cp->ctx2) vsa_ctx_destroy(cp->ctx2);
            cp->ctx2 = nullptr;
            leave(scratch);
            return VSA_HS_NOMEM;
        }
    }
    vsa_ctx_t *cx[2] = {scratch->ctx, cp->ctx2 ? cp->ctx2 : scratch->ctx};
    const vsa_plan_t *pl[2] = {cp->plan, cp->plan2 ? cp->plan2 : cp->plan};
    struct Buf {
        uint64_t *k = nullptr;
        uint32_t *i = nullptr;
        uint64_t cap = 0;
    } buf[2];
    auto grow = [&](Buf &b, uint64_t n) -> bool {
        if (n <= b.cap) return true;
        vsa::host_pinned_free(b.k);
        vsa::host_pinned_free(b.i);
        b.cap = n + n / 4 + 1024;
        b.k = (uint64_t *)vsa::host_pinned_alloc(b.cap * 8);
        b.i = (uint32_t *)vsa::host_pinned_alloc(b.cap * 4);
        return b.k && b.i;
    };
    static const bool timing = getenv("VSA_HOST_TIMING") != nullptr;
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point a, clk::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    /* hsbench's repeat loop, pipelined two passes deep: the scans of passes
     * k + 1 and k + 2 are queued on the GPU before the host replays pass k.
     * Pass k's records are copied on its context's copy stream after pass
     * k's scan (records_mark), beside scan k + 1; scan k + 2 (same context,
     * same result buffers) waits for that copy on the device.  The GPU never
     * waits for the host while a pass is queued ahead, and the copies leave
     * the scan stream (they sat between the scans: ~0.1 ms of 0.93 ms per
     * 4 GiB pass). */
    uint64_t launches_at[2] = {0, 0};
    auto queue = [&](uint32_t k) -> int {
        uint64_t dummy = 0;
        vsa_ctx_t *c = cx[k & 1];
        if (vsa_scan_plan(c, ddb, pl[k & 1], VSA_SCAN_ASYNC, &dummy) != VSA_OK ||
            vsa::records_mark(c) != VSA_OK)
            return VSA_HS_UNKNOWN_ERROR;
        launches_at[k & 1] = vsa_scan_launches(c);
        return VSA_HS_SUCCESS;
    };
    rc = queue(0);
    if (rc == VSA_HS_SUCCESS && repeats > 1) rc = queue(1);
    for (uint32_t k = 0; k < repeats && rc == VSA_HS_SUCCESS; k++) {
        vsa_ctx_t *c = cx[k & 1];
        Buf &b = buf[k & 1];
        const auto t0 = clk::now();
        uint64_t nm = 0;
        /* pass k complete (its count published; an overflow rescans here),
         * its records copied behind the scan queued after it, then pass
         * k + 2 on the same context behind that copy */
        /* a rescan inside the wait (an overflow) ran after the mark */
        if (vsa_scan_wait(c, &nm) != VSA_OK || !grow(b, nm) ||
            vsa::records_fetch_async(c, nm, b.k, b.i,
                                     vsa_scan_launches(c) != launches_at[k & 1]) != VSA_OK) {
            rc = VSA_HS_UNKNOWN_ERROR;
            break;
        }
        if (k + 2 < repeats && (rc = queue(k + 2)) != VSA_HS_SUCCESS) break;
        if (vsa::records_wait(c) != VSA_OK) {
            rc = VSA_HS_UNKNOWN_ERROR;
            break;
        }
        const auto t1 = clk::now();
        const bool last = k + 1 == repeats;
        rc = corpus_replay(cp, b.k, b.i, nm, last ? counts : nullptr, last ? digests : nullptr,
                           &totals[k], threads);
        if (timing)
            fprintf(stderr, "vsa_hs_corpus_scan_repeats: pass %u wait+copy %.3f ms, replay %.3f ms "
                    "(%llu records)\n", k, ms(t0, t1), ms(t1, clk::now()),
                    (unsigned long long)nm);
    }
    /* passes still queued after a failure complete before the buffers go */
    for (vsa_ctx_t *c : cx) (void)vsa_scan_wait(c, nullptr);
    for (vsa_ctx_t *c : cx) (void)vsa_sync(c);
    for (Buf &b : buf) {
        vsa::host_pinned_free(b.k);
        vsa::host_pinned_free(b.i);
    }
    leave(scratch);
    return rc;
}

int vsa_hs_scan_corpus(const vsa_hs_database_t *db, vsa_hs_scratch_t *scratch,
                       const uint8_t *d_data, const uint8_t *h_data, const uint64_t *offsets,
                       const uint64_t *lens, const uint32_t *stream_ids, uint32_t nblocks,
                       uint64_t *counts, uint64_t *total, unsigned threads) {
    if (!total) return VSA_HS_INVALID;
    vsa_hs_corpus_t *c = nullptr;
    int rc = vsa_hs_corpus_prepare(db, scratch, d_data, h_data, offsets, lens, stream_ids,
                                   nblocks, &c);
    if (rc != VSA_HS_SUCCESS) return rc;
    rc = vsa_hs_corpus_scan(c, counts, total, threads);
    vsa_hs_corpus_free(c);
    return rc;
}

/* runtime.c:545-575 */
int vsa_hs_open_stream(const vsa_hs_database_t *db, unsigned int flags,
                       vsa_hs_stream_t **stream) {
    (void)flags;
    if (!stream) return VSA_HS_INVALID;
    if (!valid_db(db)) return VSA_HS_INVALID;
    if (db->mode != VSA_HS_MODE_STREAM) return VSA_HS_DB_MODE_ERROR;
    vsa_hs_stream *s = new (std::nothrow) vsa_hs_stream;
    if (!s) return VSA_HS_NOMEM;
    init_stream(s, db);
    *stream = s;
    return VSA_HS_SUCCESS;
}

/* runtime.c:868-996 */
int vsa_hs_scan_stream(vsa_hs_stream_t *id, const char *data, unsigned int length,
                       unsigned int flags, vsa_hs_scratch_t *scratch,
                       vsa_hs_match_event_handler onEvent, void *ctxt) {
    (void)flags;
    if (!id || id->magic != STREAM_MAGIC || !scratch || !data) return VSA_HS_INVALID;
    int rc = enter(id->db, scratch);
    if (rc != VSA_HS_SUCCESS) return rc;
    if (id->terminated) {
        leave(scratch);
        return VSA_HS_SCAN_TERMINATED;
    }
    if (!length) {
        leave(scratch);
        return VSA_HS_SUCCESS;
    }
    const uint8_t *b = (const uint8_t *)data;
    const size_t l = length;
    rc = scan_writes(id, scratch, &b, &l, 1, onEvent, ctxt);
    leave(scratch);
    return rc;
}

/* runtime.c:999-1025: pure literal databases have no end-of-data matches */
int vsa_hs_close_stream(vsa_hs_stream_t *id, vsa_hs_scratch_t *scratch,
                        vsa_hs_match_event_handler onEvent, void *ctxt) {
    (void)ctxt;
    if (!id || id->magic != STREAM_MAGIC) return VSA_HS_INVALID;
    if (onEvent) {
        if (!scratch || scratch->magic != SCRATCH_MAGIC || !device_db(scratch, id->db))
            return VSA_HS_INVALID;
        if (scratch->in_use.load()) return VSA_HS_SCRATCH_IN_USE;
    }
    id->magic = 0;
    delete id;
    return VSA_HS_SUCCESS;
}

/* runtime.c:1028-1055 */
int vsa_hs_reset_stream(vsa_hs_stream_t *id, unsigned int flags, vsa_hs_scratch_t *scratch,
                        vsa_hs_match_event_handler onEvent, void *context) {
    (void)flags;
    (void)context;
    if (!id || id->magic != STREAM_MAGIC) return VSA_HS_INVALID;
    if (onEvent) {
        if (!scratch || scratch->magic != SCRATCH_MAGIC || !device_db(scratch, id->db))
            return VSA_HS_INVALID;
        if (scratch->in_use.load()) return VSA_HS_SCRATCH_IN_USE;
    }
    init_stream(id, id->db);
    return VSA_HS_SUCCESS;
}

/* runtime.c:740-779: no EOD matches exist in a pure-literal database, so
 * the reset reports nothing before the copy */
int vsa_hs_reset_and_copy_stream(vsa_hs_stream_t *to_id, const vsa_hs_stream_t *from_id,
                                 vsa_hs_scratch_t *scratch, vsa_hs_match_event_handler onEvent,
                                 void *context) {
    (void)context;
    if (!from_id || from_id->magic != STREAM_MAGIC || !from_id->db) return VSA_HS_INVALID;
    if (!to_id || to_id->magic != STREAM_MAGIC || to_id->db != from_id->db) return VSA_HS_INVALID;
    if (to_id == from_id) return VSA_HS_INVALID;
    if (onEvent) {
        if (!scratch || scratch->magic != SCRATCH_MAGIC || !device_db(scratch, to_id->db))
            return VSA_HS_INVALID;
        if (scratch->in_use.load()) return VSA_HS_SCRATCH_IN_USE;
    }
    to_id->offset = from_id->offset;
    to_id->hist = from_id->hist;
    to_id->exhausted = from_id->exhausted;
    to_id->terminated = from_id->terminated;
    return VSA_HS_SUCCESS;
}

/* runtime.c:713-738 */
int vsa_hs_copy_stream(vsa_hs_stream_t **to_id, const vsa_hs_stream_t *from_id) {
    if (!to_id) return VSA_HS_INVALID;
    *to_id = nullptr;
    if (!from_id || from_id->magic != STREAM_MAGIC || !from_id->db) return VSA_HS_INVALID;
    vsa_hs_stream *s = new (std::nothrow) vsa_hs_stream;
    if (!s) return VSA_HS_NOMEM;
    s->db = from_id->db;
    s->offset = from_id->offset;
    s->hist = from_id->hist;
    s->exhausted = from_id->exhausted;
    s->terminated = from_id->terminated;
    *to_id = s;
    return VSA_HS_SUCCESS;
}

/* hs_stream_size, hs_common.h:183: the bytes of one open stream's state */
int vsa_hs_stream_size(const vsa_hs_database_t *db, size_t *stream_size) {
    if (!stream_size || !valid_db(db)) return VSA_HS_INVALID;
    if (db->mode != VSA_HS_MODE_STREAM) return VSA_HS_DB_MODE_ERROR;
    *stream_size = sizeof(vsa_hs_stream) + db->max_len + HIST_MIN + db->n_ekeys;
    return VSA_HS_SUCCESS;
}

/* scratch.c:373-423 (hs_clone_scratch): a new scratch, with its own GPU
 * context, serving the same databases */
int vsa_hs_clone_scratch(const vsa_hs_scratch_t *src, vsa_hs_scratch_t **dest) {
    if (!dest || !src || src->magic != SCRATCH_MAGIC) return VSA_HS_INVALID;
    *dest = nullptr;
    vsa_hs_scratch *s = new (std::nothrow) vsa_hs_scratch;
    if (!s) return VSA_HS_NOMEM;
    /* the source's GPU, whatever VSA_DEVICE says now */
    if (!src->ctx || vsa_ctx_create(vsa::ctxDevice(src->ctx), &s->ctx) != VSA_OK) {
        delete s;
        return VSA_HS_NOMEM;
    }
    for (const auto &e : src->dbs) {
        const uint8_t *blob = nullptr;
        size_t size = 0;
        vsa_db_t *d = nullptr;
        if (vsa::dbHostBlob(e.second, &blob, &size) != VSA_OK ||
            vsa_db_load(s->ctx, blob, size, &d) != VSA_OK) {
            vsa_hs_free_scratch(s);
            return VSA_HS_NOMEM;
        }
        s->dbs.emplace_back(e.first, d);
    }
    *dest = s;
    return VSA_HS_SUCCESS;
}

/* hs_scratch_size, hs_runtime.h:593: host bytes of the scratch and of the
 * database copies it holds (their device copies mirror them) */
int vsa_hs_scratch_size(const vsa_hs_scratch_t *scratch, size_t *scratch_size) {
    if (!scratch_size || !scratch || scratch->magic != SCRATCH_MAGIC) return VSA_HS_INVALID;
    size_t n = sizeof(vsa_hs_scratch);
    for (const auto &e : scratch->dbs) {
        const uint8_t *blob = nullptr;
        size_t size = 0;
        if (vsa::dbHostBlob(e.second, &blob, &size) == VSA_OK) n += size;
    }
    *scratch_size = n;
    return VSA_HS_SUCCESS;
}

/* hs_valid_platform, hs_common.h:463: the GPU path needs no host ISA level */
int vsa_hs_valid_platform(void) { return VSA_HS_SUCCESS; }

/* hs_version, hs_common.h:446 (HS_VERSION_STRING: "major.minor.patch date") */
const char *vsa_hs_version(void) { return "5.4.11 vectorscan_amd gfx950"; }

/* ------------------------------------------------------ serialization --
 * The reference's serialized database (database.c:61-110, db_decode_header
 * :122-170): 32 header bytes -- magic 0xdbdbdbdb, version (HS_VERSION_32BIT
 * of 5.4.11), bytecode length, platform (u64, unaligned at byte 12), CRC-32C
 * of the bytecode, two reserved words -- then the bytecode, then zeroes up to
 * sizeof(struct hs_database) (104) + length bytes in all.
 *
 * The bytecode starts with the fields of struct RoseEngine that the
 * reference reads without running it (rose_internal.h:330-345): pureLiteral
 * = 1, runtimeImpl = ROSE_RUNTIME_PURE_LITERAL, canExhaust, hasSom, mode at
 * byte 12 (hs_serialized_database_info reads it there), historyRequired.
 * The rest is this engine's own: tag "VSAL", a format version, the compile
 * mode and the patterns as given (id, flags, length, bytes); deserializing
 * compiles them again (deterministic: the same HWLM blob).  A database
 * serialized by the reference holds a full RoseEngine instead and is refused
 * with HS_DB_PLATFORM_ERROR; the envelope, version and CRC checks are the
 * reference's. */
} // extern "C"
namespace {
constexpr uint32_t HS_DB_MAGIC = 0xdbdbdbdbu;
constexpr uint32_t HS_DB_VERSION = (5u << 24) | (4u << 16) | (11u << 8);
constexpr size_t HS_DB_HEADER = 104; /* sizeof(struct hs_database), database.h:103-114 */
constexpr size_t HS_DB_FIELDS = 32;  /* the header words database.c serializes */
/* HS_PLATFORM_NOAVX2 | NOAVX512 | NOAVX512VBMI (database.h:55-57): no host
 * SIMD level is assumed */
constexpr uint64_t VSA_PLATFORM = (4ull << 13) | (8ull << 13) | (0x10ull << 13);
constexpr uint32_t VSAL_TAG = 0x4c415356u; /* "VSAL" */
constexpr uint32_t VSAL_FORMAT = 1;
constexpr size_t VSAL_OFF = 64; /* our section, after the RoseEngine prefix */

/* CRC-32C as Crc32c_ComputeBuf(0, ...) (crc32.c:528-601: reflected
 * polynomial 0x82F63B78, no pre- or post-inversion) */
uint32_t crc32c(const uint8_t *p, size_t n) {
    static uint32_t T[256];
    static std::once_flag once;
    std::call_once(once, [] {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
            T[i] = c;
        }
    });
    uint32_t crc = 0;
    while (n--) crc = T[(crc ^ *p++) & 0xff] ^ (crc >> 8);
    return crc;
}

void put32(std::vector<uint8_t> &b, size_t off, uint32_t v) { memcpy(b.data() + off, &v, 4); }
uint32_t get32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}

std::vector<uint8_t> bytecode_of(const vsa_hs_database *db) {
    size_t n = VSAL_OFF + 16;
    for (const auto &x : db->src) n += 12 + x.e.size();
    std::vector<uint8_t> b(n, 0);
    bool exhaust = !db->pats.empty(), som = false;
    for (const auto &pt : db->pats) {
        exhaust &= pt.ekey != NO_EKEY;
        som |= pt.som;
    }
    b[0] = 1;               /* pureLiteral */
    b[4] = 1;               /* runtimeImpl: ROSE_RUNTIME_PURE_LITERAL */
    b[6] = exhaust ? 1 : 0; /* canExhaust */
    b[7] = som ? 1 : 0;     /* hasSom */
    put32(b, 12, db->mode);
    put32(b, 16, db->mode == VSA_HS_MODE_BLOCK ? 0u : (uint32_t)db->max_len);
    put32(b, VSAL_OFF, VSAL_TAG);
    put32(b, VSAL_OFF + 4, VSAL_FORMAT);
    put32(b, VSAL_OFF + 8, db->mode_full);
    put32(b, VSAL_OFF + 12, (uint32_t)db->src.size());
    size_t o = VSAL_OFF + 16;
    for (const auto &x : db->src) {
        put32(b, o, x.id);
        put32(b, o + 4, x.flags);
        put32(b, o + 8, (uint32_t)x.e.size());
        memcpy(b.data() + o + 12, x.e.data(), x.e.size());
        o += 12 + x.e.size();
    }
    return b;
}

/* db_decode_header (database.c:122-170) + the platform check (:117-120) */
int decode_header(const char *bytes, size_t length, uint32_t *version, uint64_t *platform,
                  const uint8_t **code, uint32_t *code_len) {
    if (!bytes || length < HS_DB_HEADER) return VSA_HS_INVALID;
    const uint8_t *p = (const uint8_t *)bytes;
    if (get32(p) != HS_DB_MAGIC) return VSA_HS_INVALID;
    *version = get32(p + 4);
    if (*version != HS_DB_VERSION) return VSA_HS_DB_VERSION_ERROR;
    *code_len = get32(p + 8);
    if (length != HS_DB_HEADER + *code_len) return VSA_HS_INVALID;
    memcpy(platform, p + 12, 8);
    *code = p + HS_DB_FIELDS;
    return VSA_HS_SUCCESS;
}
} // namespace
extern "C" {

/* hs_serialize_database, hs_common.h:104 (database.c:61-110) */
int vsa_hs_serialize_database(const vsa_hs_database_t *db, char **bytes, size_t *length) {
    if (!db || !bytes || !length) return VSA_HS_INVALID;
    if (!valid_db(db)) return VSA_HS_INVALID;
    const std::vector<uint8_t> code = bytecode_of(db);
    const size_t n = HS_DB_HEADER + code.size();
    char *out = (char *)malloc(n);
    if (!out) return VSA_HS_NOMEM;
    memset(out, 0, n);
    const uint32_t hdr[3] = {HS_DB_MAGIC, HS_DB_VERSION, (uint32_t)code.size()};
    memcpy(out, hdr, 12);
    memcpy(out + 12, &VSA_PLATFORM, 8);
    const uint32_t crc = crc32c(code.data(), code.size());
    memcpy(out + 20, &crc, 4); /* reserved0 / reserved1 stay 0 */
    memcpy(out + HS_DB_FIELDS, code.data(), code.size());
    *bytes = out;
    *length = n;
    return VSA_HS_SUCCESS;
}

/* hs_deserialize_database, hs_common.h:133 (database.c:246-296) */
int vsa_hs_deserialize_database(const char *bytes, size_t length, vsa_hs_database_t **db) {
    if (!bytes || !db) return VSA_HS_INVALID;
    *db = nullptr;
    uint32_t version, code_len;
    uint64_t platform;
    const uint8_t *code;
    int r = decode_header(bytes, length, &version, &platform, &code, &code_len);
    if (r != VSA_HS_SUCCESS) return r;
    /* the order of database.c:246-296: platform, then CRC; then this
     * engine's tag (a reference RoseEngine has none) */
    if (platform != VSA_PLATFORM) return VSA_HS_DB_PLATFORM_ERROR;
    uint32_t crc;
    memcpy(&crc, bytes + 20, 4);
    if (crc32c(code, code_len) != crc) return VSA_HS_INVALID;
    if (code_len < VSAL_OFF + 16 || get32(code + VSAL_OFF) != VSAL_TAG ||
        get32(code + VSAL_OFF + 4) != VSAL_FORMAT)
        return VSA_HS_DB_PLATFORM_ERROR;
    const unsigned mode = get32(code + VSAL_OFF + 8), n = get32(code + VSAL_OFF + 12);
    std::vector<std::string> es;
    std::vector<unsigned> fl, ids;
    std::vector<size_t> lens;
    size_t o = VSAL_OFF + 16;
    for (unsigned i = 0; i < n; i++) {
        if (o + 12 > code_len) return VSA_HS_INVALID;
        ids.push_back(get32(code + o));
        fl.push_back(get32(code + o + 4));
        const uint32_t len = get32(code + o + 8);
        if (o + 12 + len > code_len) return VSA_HS_INVALID;
        es.emplace_back((const char *)code + o + 12, len);
        lens.push_back(len);
        o += 12 + len;
    }
    std::vector<const char *> ep;
    for (const auto &e : es) ep.push_back(e.c_str());
    vsa_hs_compile_error_t *err = nullptr;
    r = vsa_hs_compile_lit_multi(ep.data(), fl.data(), ids.data(), lens.data(), n, mode, nullptr,
                                 db, &err);
    if (r != VSA_HS_SUCCESS) {
        vsa_hs_free_compile_error(err);
        return VSA_HS_INVALID;
    }
    return VSA_HS_SUCCESS;
}

/* hs_serialized_database_size, hs_common.h:226 (database.c:316-332) */
int vsa_hs_serialized_database_size(const char *bytes, size_t length, size_t *deserialized_size) {
    uint32_t version, code_len;
    uint64_t platform;
    const uint8_t *code;
    int r = decode_header(bytes, length, &version, &platform, &code, &code_len);
    if (r != VSA_HS_SUCCESS) return r;
    if (!deserialized_size) return VSA_HS_INVALID;
    *deserialized_size = HS_DB_HEADER + code_len;
    return VSA_HS_SUCCESS;
}

/* hs_database_size, hs_common.h:199 (database.c:300-312): the size of the
 * database in the reference's layout (header + bytecode) */
int vsa_hs_database_size(const vsa_hs_database_t *db, size_t *database_size) {
    if (!database_size) return VSA_HS_INVALID;
    if (!valid_db(db)) return VSA_HS_INVALID;
    *database_size = HS_DB_HEADER + bytecode_of(db).size();
    return VSA_HS_SUCCESS;
}

} // extern "C"
namespace {
/* print_database_string (database.c:358-416) */
int database_string(char **info, uint32_t version, uint64_t plat, uint32_t mode) {
    const char *features = (plat & (0x10ull << 13))
                               ? (plat & (8ull << 13)) ? (plat & (4ull << 13)) ? "" : "AVX2"
                                                       : "AVX512"
                               : "AVX512VBMI";
    const char *m = mode == VSA_HS_MODE_STREAM ? "STREAM"
                    : mode == VSA_HS_MODE_VECTORED ? "VECTORED" : "BLOCK";
    char buf[256];
    snprintf(buf, sizeof(buf), "Version: %u.%u.%u Features: %s Mode: %s", (version >> 24) & 0xff,
             (version >> 16) & 0xff, (version >> 8) & 0xff, features, m);
    *info = strdup(buf);
    return *info ? VSA_HS_SUCCESS : VSA_HS_NOMEM;
}
} // namespace
extern "C" {

/* hs_serialized_database_info, hs_common.h:267 (database.c:419-436): the
 * mode from the bytecode's RoseEngine.mode, whoever serialized it */
int vsa_hs_serialized_database_info(const char *bytes, size_t length, char **info) {
    if (!info) return VSA_HS_INVALID;
    *info = nullptr;
    uint32_t version, code_len;
    uint64_t platform;
    const uint8_t *code;
    int r = decode_header(bytes, length, &version, &platform, &code, &code_len);
    if (r != VSA_HS_SUCCESS) return r;
    if (code_len < 16) return VSA_HS_INVALID;
    return database_string(info, version, platform, get32(code + 12));
}

/* hs_database_info, hs_common.h:245 (database.c:438-455) */
int vsa_hs_database_info(const vsa_hs_database_t *db, char **info) {
    if (!info) return VSA_HS_INVALID;
    *info = nullptr;
    if (!valid_db(db)) return VSA_HS_INVALID;
    return database_string(info, HS_DB_VERSION, VSA_PLATFORM, db->mode);
}

} // extern "C"
