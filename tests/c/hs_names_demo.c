/*
 * A program written against the reference's hs API (hs_compile_lit_multi,
 * hs_alloc_scratch, hs_scan, streams, hs_scan_vector, serialization; the
 * names of hs_common.h / hs_compile.h / hs_runtime.h), built on
 * include/vectorscan_amd_hs_names.h instead of <hs.h>.  It checks every
 * result against a brute-force scan of its own buffer: the (to, id) match
 * set of each literal (caseless, SINGLEMATCH), the same set from a stream
 * cut into writes and from a vectored scan of the same pieces, and from a
 * serialized / deserialized copy of the database.  Prints "hs_names_demo:
 * ... OK" and exits 0 when all agree.
 *   tests/c/hs_names_demo [bytes]
 */
#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vectorscan_amd_hs_names.h"

typedef struct {
    unsigned long long *to;
    unsigned *id;
    size_t n, cap;
} Matches;

static int on_match(unsigned int id, unsigned long long from, unsigned long long to,
                    unsigned int flags, void *ctx) {
    (void)from;
    (void)flags;
    Matches *m = (Matches *)ctx;
    if (m->n == m->cap) {
        m->cap = m->cap ? 2 * m->cap : 1024;
        m->to = (unsigned long long *)realloc(m->to, m->cap * sizeof(*m->to));
        m->id = (unsigned *)realloc(m->id, m->cap * sizeof(*m->id));
    }
    m->to[m->n] = to;
    m->id[m->n] = id;
    m->n++;
    return 0;
}

static int cmp_pair(const void *a, const void *b) {
    const unsigned long long *x = (const unsigned long long *)a, *y = (const unsigned long long *)b;
    return x[0] < y[0] ? -1 : x[0] > y[0] ? 1 : x[1] < y[1] ? -1 : x[1] > y[1];
}

/* the match set as sorted (to, id) pairs */
static unsigned long long *pairs(const Matches *m) {
    unsigned long long *p = (unsigned long long *)malloc((m->n + 1) * 2 * sizeof(*p));
    for (size_t i = 0; i < m->n; i++) {
        p[2 * i] = m->to[i];
        p[2 * i + 1] = m->id[i];
    }
    qsort(p, m->n, 2 * sizeof(*p), cmp_pair);
    return p;
}

static int same(const char *what, const Matches *got, const Matches *want) {
    if (got->n != want->n) {
        printf("hs_names_demo: %s: %zu matches, brute force %zu\n", what, got->n, want->n);
        return 0;
    }
    unsigned long long *a = pairs(got), *b = pairs(want);
    const int eq = memcmp(a, b, got->n * 2 * sizeof(*a)) == 0;
    if (!eq) printf("hs_names_demo: %s: match sets differ\n", what);
    free(a);
    free(b);
    return eq;
}

#define NPAT 5
static const char *pats[NPAT] = {"foobar", "Hello", "abcab", "zq", "needle"};
static const unsigned flags[NPAT] = {0, HS_FLAG_CASELESS, 0, HS_FLAG_SINGLEMATCH, 0};
static const unsigned ids[NPAT] = {10, 20, 30, 40, 50};

/* every end of every literal (abcab overlaps itself), SINGLEMATCH: the first */
static void brute(const char *buf, size_t n, Matches *m) {
    for (int p = 0; p < NPAT; p++) {
        const size_t L = strlen(pats[p]);
        for (size_t e = L; e <= n; e++) {
            const char *s = buf + e - L;
            int ok = 1;
            for (size_t k = 0; k < L && ok; k++)
                ok = (flags[p] & HS_FLAG_CASELESS) ? tolower((unsigned char)s[k]) ==
                                                         tolower((unsigned char)pats[p][k])
                                                   : s[k] == pats[p][k];
            if (ok) {
                on_match(ids[p], 0, e, 0, m);
                if (flags[p] & HS_FLAG_SINGLEMATCH) break;
            }
        }
    }
}

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? (size_t)strtoull(argv[1], NULL, 0) : (4u << 20);
    char *buf = (char *)malloc(n);
    unsigned long long rs = 0x9e3779b97f4a7c15ULL;
    for (size_t i = 0; i < n; i++) {
        rs ^= rs << 13;
        rs ^= rs >> 7;
        rs ^= rs << 17;
        buf[i] = "abcdefghijklmnopqrstuvwxyzHELO"[rs % 30];
    }
    for (size_t i = 0; i + 64 < n; i += 4093) { /* planted occurrences */
        const char *p = pats[(i / 4093) % NPAT];
        memcpy(buf + i, p, strlen(p));
        if ((i / 4093) % 7 == 0) memcpy(buf + i + 10, "hElLo", 5);
    }
    size_t lens[NPAT];
    for (int p = 0; p < NPAT; p++) lens[p] = strlen(pats[p]);

    Matches want = {NULL, NULL, 0, 0};
    brute(buf, n, &want);
    int ok = 1;

    /* block mode */
    hs_database_t *db = NULL;
    hs_compile_error_t *err = NULL;
    if (hs_compile_lit_multi(pats, flags, ids, lens, NPAT, HS_MODE_BLOCK, NULL, &db, &err) !=
        HS_SUCCESS) {
        printf("hs_names_demo: compile failed: %s\n", err ? err->message : "?");
        hs_free_compile_error(err);
        return 1;
    }
    hs_scratch_t *scratch = NULL;
    if (hs_alloc_scratch(db, &scratch) != HS_SUCCESS) return 1;
    Matches got = {NULL, NULL, 0, 0};
    if (hs_scan(db, buf, (unsigned)n, 0, scratch, on_match, &got) != HS_SUCCESS) return 1;
    ok = same("hs_scan", &got, &want) && ok;

    /* a serialized copy scans the same */
    char *bytes = NULL;
    size_t blen = 0;
    hs_database_t *db2 = NULL;
    if (hs_serialize_database(db, &bytes, &blen) != HS_SUCCESS ||
        hs_deserialize_database(bytes, blen, &db2) != HS_SUCCESS)
        return 1;
    free(bytes);
    hs_scratch_t *scratch2 = NULL;
    if (hs_alloc_scratch(db2, &scratch2) != HS_SUCCESS) return 1;
    Matches got2 = {NULL, NULL, 0, 0};
    if (hs_scan(db2, buf, (unsigned)n, 0, scratch2, on_match, &got2) != HS_SUCCESS) return 1;
    ok = same("hs_scan (deserialized)", &got2, &want) && ok;

    /* stream mode: the buffer as writes of 1,000 bytes (literals span them) */
    hs_database_t *sdb = NULL;
    if (hs_compile_lit_multi(pats, flags, ids, lens, NPAT, HS_MODE_STREAM, NULL, &sdb, &err) !=
        HS_SUCCESS)
        return 1;
    hs_scratch_t *sscratch = NULL;
    if (hs_alloc_scratch(sdb, &sscratch) != HS_SUCCESS) return 1;
    hs_stream_t *st = NULL;
    if (hs_open_stream(sdb, 0, &st) != HS_SUCCESS) return 1;
    Matches sgot = {NULL, NULL, 0, 0};
    for (size_t off = 0; off < n; off += 1000) {
        const size_t w = n - off < 1000 ? n - off : 1000;
        if (hs_scan_stream(st, buf + off, (unsigned)w, 0, sscratch, on_match, &sgot) != HS_SUCCESS)
            return 1;
    }
    if (hs_close_stream(st, sscratch, on_match, &sgot) != HS_SUCCESS) return 1;
    ok = same("hs_scan_stream", &sgot, &want) && ok;

    /* vectored mode: the same pieces in one call */
    hs_database_t *vdb = NULL;
    if (hs_compile_lit_multi(pats, flags, ids, lens, NPAT, HS_MODE_VECTORED, NULL, &vdb, &err) !=
        HS_SUCCESS)
        return 1;
    hs_scratch_t *vscratch = NULL;
    if (hs_alloc_scratch(vdb, &vscratch) != HS_SUCCESS) return 1;
    const unsigned npieces = (unsigned)((n + 99999) / 100000);
    const char **data = (const char **)malloc(npieces * sizeof(*data));
    unsigned *plen = (unsigned *)malloc(npieces * sizeof(*plen));
    for (unsigned i = 0; i < npieces; i++) {
        data[i] = buf + (size_t)i * 100000;
        plen[i] = (unsigned)(n - (size_t)i * 100000 < 100000 ? n - (size_t)i * 100000 : 100000);
    }
    Matches vgot = {NULL, NULL, 0, 0};
    if (hs_scan_vector(vdb, data, plen, npieces, 0, vscratch, on_match, &vgot) != HS_SUCCESS)
        return 1;
    ok = same("hs_scan_vector", &vgot, &want) && ok;

    hs_free_scratch(scratch);
    hs_free_scratch(scratch2);
    hs_free_scratch(sscratch);
    hs_free_scratch(vscratch);
    hs_free_database(db);
    hs_free_database(db2);
    hs_free_database(sdb);
    hs_free_database(vdb);
    printf("hs_names_demo: %zu bytes, %zu matches (%s) %s\n", n, want.n, hs_version(),
           ok ? "OK" : "MISMATCH");
    return ok ? 0 : 1;
}
