/*
 * dropin_threads.c — measurement tool (verdict r03 item 6): small hwlmExec
 * calls from T POSIX threads (no interpreter lock), three ways, same blob and
 * bytes:
 *   gpu      the drop-in hwlmExec (registered blob, one launch per call, each
 *            thread its own context: include/vectorscan_amd.h part 1)
 *   batcher  vsa_batcher_hwlmExec (concurrent calls share one launch)
 *   cpu      the oracle's SSE2 port of the reference FDR loop (oracle.c
 *            orc_fdr_exec_simd, the CPU baseline engine), one call per call
 * for T in 1..32 and buffers of 1 KiB-4 MiB; each cell runs `secs` seconds.
 * Database: 5,000 random printable literals of 4-8 bytes (2 % nocase, the
 * cfg-4 shape); corpus: 64 MiB printable with one planted literal per
 * 64 KiB.  One JSON line per (mode, threads, bytes): calls/s, GB/s, mean /
 * p50 / p99 call latency, matches per call.  The oracle is linked only as
 * the CPU comparator.
 *   dropin_threads [secs] [max_threads]
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "vectorscan_amd.h"

#define ALL_GROUPS (~0ULL)

typedef struct {
    uint64_t end;
    uint32_t id;
} orc_match;
long orc_fdr_exec_simd(const void *eng, const uint8_t *buf, size_t len, size_t start,
                       uint64_t groups, orc_match *out, size_t cap, int *status);

static uint64_t rs = 0x9e3779b97f4a7c15ULL;
static uint32_t rnd(void) {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return (uint32_t)(rs >> 11);
}

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static __thread uint64_t t_matches;
static hwlmcb_rv_t count_cb(size_t end, uint32_t id, struct hs_scratch *s) {
    (void)end;
    (void)id;
    (void)s;
    t_matches++;
    return ALL_GROUPS;
}

enum { M_GPU, M_BATCH, M_CPU };
static const char *mode_name[] = {"gpu", "batcher", "cpu"};

static const uint8_t *g_corpus;
static size_t g_corpus_len;
static void *g_blob;
static const void *g_eng;
static vsa_batcher_t *g_bat;
static volatile int g_go, g_stop;

#define MAX_LAT 200000
typedef struct {
    int mode, t;
    size_t size;
    uint64_t calls, matches, errors;
    float *lat; /* us */
    orc_match *out;
} job_t;

static void *worker(void *p) {
    job_t *j = (job_t *)p;
    size_t off = ((size_t)j->t * 7919 * 1024) % (g_corpus_len - j->size);
    while (!g_go) {
    }
    while (!g_stop) {
        const uint8_t *buf = g_corpus + off;
        off += j->size + 64;
        if (off + j->size > g_corpus_len) off = (size_t)(j->t * 64);
        const double t0 = now();
        t_matches = 0;
        int rc = 0;
        if (j->mode == M_GPU) {
            rc = hwlmExec((const struct HWLM *)g_blob, buf, j->size, 0, count_cb, NULL,
                          ALL_GROUPS);
        } else if (j->mode == M_BATCH) {
            rc = vsa_batcher_hwlmExec(g_bat, (const struct HWLM *)g_blob, buf, j->size, 0,
                                      count_cb, NULL, ALL_GROUPS);
        } else {
            int st = 0;
            t_matches = (uint64_t)orc_fdr_exec_simd(g_eng, buf, j->size, 0, ~0ULL, j->out, 4096,
                                                    &st);
            rc = st;
        }
        const double dt = now() - t0;
        if (rc) j->errors++;
        if (j->calls < MAX_LAT) j->lat[j->calls] = (float)(dt * 1e6);
        j->calls++;
        j->matches += t_matches;
    }
    return NULL;
}

static int cmpf(const void *a, const void *b) {
    const float x = *(const float *)a, y = *(const float *)b;
    return x < y ? -1 : x > y;
}

static void cell(int mode, int threads, size_t size, double secs) {
    job_t jobs[64];
    pthread_t th[64];
    g_go = 0;
    g_stop = 0;
    for (int t = 0; t < threads; t++) {
        jobs[t] = (job_t){mode, t, size, 0, 0, 0, malloc(MAX_LAT * sizeof(float)),
                          malloc(4096 * sizeof(orc_match))};
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    const double t0 = now();
    g_go = 1;
    while (now() - t0 < secs) {
        struct timespec ts = {0, 2000000};
        nanosleep(&ts, NULL);
    }
    g_stop = 1;
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    const double el = now() - t0;
    uint64_t calls = 0, matches = 0, errors = 0, nl = 0;
    for (int t = 0; t < threads; t++) {
        calls += jobs[t].calls;
        matches += jobs[t].matches;
        errors += jobs[t].errors;
        nl += jobs[t].calls < MAX_LAT ? jobs[t].calls : MAX_LAT;
    }
    float *all = malloc((nl + 1) * sizeof(float));
    uint64_t k = 0;
    double sum = 0;
    for (int t = 0; t < threads; t++) {
        const uint64_t n = jobs[t].calls < MAX_LAT ? jobs[t].calls : MAX_LAT;
        for (uint64_t i = 0; i < n; i++) {
            all[k++] = jobs[t].lat[i];
            sum += jobs[t].lat[i];
        }
        free(jobs[t].lat);
        free(jobs[t].out);
    }
    qsort(all, k, sizeof(float), cmpf);
    uint64_t launches = 0, served = 0;
    if (mode == M_BATCH) vsa_batcher_stats(g_bat, &launches, &served);
    printf("{\"mode\": \"%s\", \"threads\": %d, \"bytes\": %zu, \"calls_per_s\": %.0f, "
           "\"GBps\": %.4f, \"mean_us\": %.2f, \"p50_us\": %.2f, \"p99_us\": %.2f, "
           "\"matches_per_call\": %.3f, \"errors\": %llu",
           mode_name[mode], threads, size, calls / el, calls * (double)size / el / 1e9,
           k ? sum / k : 0.0, k ? all[k / 2] : 0.0f, k ? all[(k * 99) / 100] : 0.0f,
           calls ? (double)matches / calls : 0.0, (unsigned long long)errors);
    if (mode == M_BATCH)
        printf(", \"batcher_launches_total\": %llu, \"batcher_calls_total\": %llu",
               (unsigned long long)launches, (unsigned long long)served);
    printf("}\n");
    fflush(stdout);
    free(all);
}

int main(int argc, char **argv) {
    const double secs = argc > 1 ? atof(argv[1]) : 0.3;
    const int max_t = argc > 2 ? atoi(argv[2]) : 32;
    /* the literal set */
    enum { NL = 5000 };
    static uint8_t text[NL][8];
    static vsa_literal_t lits[NL];
    for (int i = 0; i < NL; i++) {
        const int len = 4 + (int)(rnd() % 5);
        for (int k = 0; k < len; k++) text[i][k] = (uint8_t)(0x20 + rnd() % 95);
        lits[i] = (vsa_literal_t){text[i], (uint32_t)len, (uint32_t)i, (rnd() % 50) == 0, 0,
                                  0, 0, ALL_GROUPS, NULL, NULL};
    }
    vsa_build_opts_t o;
    vsa_build_opts_default(&o);
    size_t bsz = 0;
    if (vsa_hwlm_build(lits, NL, &o, &g_blob, &bsz) != 0) {
        fprintf(stderr, "build failed\n");
        return 1;
    }
    g_eng = (const uint8_t *)g_blob + 192; /* the engine after ROUNDUP_CL(sizeof(HWLM)) */
    vsa_hwlm_register(g_blob, -1);
    g_corpus_len = 64u << 20;
    uint8_t *c = malloc(g_corpus_len);
    for (size_t i = 0; i < g_corpus_len; i++) c[i] = (uint8_t)(0x20 + rnd() % 95);
    for (size_t p = 0; p + 64 < g_corpus_len; p += 64 << 10) {
        const int w = (int)(rnd() % NL);
        memcpy(c + p + rnd() % 60000, text[w], lits[w].len);
    }
    g_corpus = c;
    if (vsa_batcher_create(0, 256, 30, &g_bat) != 0) {
        fprintf(stderr, "batcher failed\n");
        return 1;
    }
    static const size_t sizes[] = {1 << 10, 4 << 10, 16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20};
    static const int tcount[] = {1, 2, 4, 8, 16, 32};
    /* warm every path (contexts, device tables, clocks) */
    for (int m = 0; m < 3; m++) cell(m, 4, 4096, 0.2);
    for (size_t s = 0; s < sizeof(sizes) / sizeof(sizes[0]); s++)
        for (size_t ti = 0; ti < sizeof(tcount) / sizeof(tcount[0]); ti++) {
            if (tcount[ti] > max_t) continue;
            for (int m = 0; m < 3; m++) cell(m, tcount[ti], sizes[s], secs);
        }
    vsa_batcher_destroy(g_bat);
    return 0;
}
