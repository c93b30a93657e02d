/*
 * abi_harness.c — TEST ONLY.  A plain C caller of libvectorscan_amd.so's
 * pointer-returning drop-ins through their real reference signatures
 * (include/vectorscan_amd.h): masks travel as __m128i in XMM registers
 * exactly as the reference's m128 arguments (shufti.h:46-55, truffle.h:45-49,
 * vermicelli.hpp:47-95, accel.h:148).  Every result is compared with the
 * test-only oracle (oracle/oracle.c, linked as the checker) on the same
 * bytes at the same address.  Exit status 0 = all equal; prints a summary.
 */
#include <emmintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vectorscan_amd.h"

/* oracle.c (checker) */
long orc_shufti(const uint8_t *lo, const uint8_t *hi, const uint8_t *buf, size_t len);
long orc_rshufti(const uint8_t *lo, const uint8_t *hi, const uint8_t *buf, size_t len);
long orc_truffle(const uint8_t *m1, const uint8_t *m2, const uint8_t *buf, size_t len);
long orc_rtruffle(const uint8_t *m1, const uint8_t *m2, const uint8_t *buf, size_t len);
long orc_verm(uint8_t c, int nocase, int negate, int reverse, const uint8_t *buf, size_t len);
long orc_dverm(uint8_t c1, uint8_t c2, int nocase, const uint8_t *buf, size_t len);
long orc_rdverm(uint8_t c1, uint8_t c2, int nocase, const uint8_t *buf, size_t len);
long orc_dverm_masked(uint8_t c1, uint8_t c2, uint8_t m1, uint8_t m2, const uint8_t *buf,
                      size_t len);
long orc_shufti_double(const uint8_t *lo1, const uint8_t *hi1, const uint8_t *lo2,
                       const uint8_t *hi2, const uint8_t *buf, size_t len, long S, long mis);
long orc_run_accel(const uint8_t *aux, const uint8_t *c, size_t len);

static uint64_t rs = 0x243f6a8885a308d3ULL;
static uint32_t rnd(void) {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return (uint32_t)(rs >> 11);
}

static long checks, fails;
static void check(const char *what, long got, long want, size_t len) {
    checks++;
    if (got != want) {
        fails++;
        if (fails < 20) fprintf(stderr, "MISMATCH %s len %zu: got %ld want %ld\n", what, len, got, want);
    }
}

static __m128i m128(const uint8_t *b) { return _mm_loadu_si128((const __m128i *)b); }

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 200;
    static const size_t lens[] = {0, 1, 5, 15, 16, 17, 18, 31, 33, 63, 64, 65, 100, 257, 1000,
                                  4097, 70000};
    uint8_t *raw = malloc(70000 + 256);
    for (int round = 0; round < rounds; round++) {
        /* alphabet: a few random bytes, so classes hit at varied densities */
        uint8_t alpha[12];
        const int na = 2 + (int)(rnd() % 10);
        for (int i = 0; i < na; i++) alpha[i] = (uint8_t)rnd();
        uint8_t cls[32] = {0};
        const int ncls = 1 + (int)(rnd() % 3);
        for (int i = 0; i < ncls; i++) {
            const uint8_t ch = alpha[rnd() % na];
            cls[ch >> 3] |= (uint8_t)(1u << (ch & 7));
        }
        uint8_t lo[16], hi[16], t1[16], t2[16];
        const int sh_ok = vsa_shufti_build_masks(cls, lo, hi) >= 0;
        vsa_truffle_build_masks(cls, t1, t2);
        const uint8_t pairs[4] = {alpha[rnd() % na], alpha[rnd() % na], alpha[rnd() % na],
                                  alpha[rnd() % na]};
        uint8_t dl1[16], dh1[16], dl2[16], dh2[16];
        const int ds_ok = vsa_shufti_build_double_masks(NULL, pairs, 2, dl1, dh1, dl2, dh2) == 0;
        const size_t len = lens[rnd() % (sizeof(lens) / sizeof(lens[0]))];
        uint8_t *buf = raw + (rnd() % 64);
        for (size_t i = 0; i < len; i++) buf[i] = (rnd() % 8) ? alpha[rnd() % na] : (uint8_t)rnd();
        const uint8_t *end = buf + len;
        const uint8_t c1 = alpha[rnd() % na], c2 = alpha[rnd() % na];
        const uint8_t uc1 = (c1 >= 'a' && c1 <= 'z') ? c1 - 32 : c1;

        if (sh_ok) {
            check("shuftiExec", shuftiExec(m128(lo), m128(hi), buf, end) - buf,
                  orc_shufti(lo, hi, buf, len), len);
            check("rshuftiExec", rshuftiExec(m128(lo), m128(hi), buf, end) - buf,
                  orc_rshufti(lo, hi, buf, len), len);
        }
        check("truffleExec", truffleExec(m128(t1), m128(t2), buf, end) - buf,
              orc_truffle(t1, t2, buf, len), len);
        check("rtruffleExec", rtruffleExec(m128(t1), m128(t2), buf, end) - buf,
              orc_rtruffle(t1, t2, buf, len), len);
        check("vermicelliExec", vermicelliExec((char)c1, 0, buf, end) - buf,
              orc_verm(c1, 0, 0, 0, buf, len), len);
        check("vermicelliExec nocase", vermicelliExec((char)uc1, 1, buf, end) - buf,
              orc_verm(uc1, 1, 0, 0, buf, len), len);
        check("nvermicelliExec", nvermicelliExec((char)c1, 0, buf, end) - buf,
              orc_verm(c1, 0, 1, 0, buf, len), len);
        check("rvermicelliExec", rvermicelliExec((char)c1, 0, buf, end) - buf,
              orc_verm(c1, 0, 0, 1, buf, len), len);
        check("rnvermicelliExec", rnvermicelliExec((char)c1, 0, buf, end) - buf,
              orc_verm(c1, 0, 1, 1, buf, len), len);
        check("vermicelliDoubleExec", vermicelliDoubleExec((char)c1, (char)c2, 0, buf, end) - buf,
              orc_dverm(c1, c2, 0, buf, len), len);
        check("rvermicelliDoubleExec",
              rvermicelliDoubleExec((char)c1, (char)c2, 0, buf, end) - buf,
              orc_rdverm(c1, c2, 0, buf, len), len);
        const uint8_t m1 = (uint8_t)(rnd() | 0x0f), m2 = (uint8_t)(rnd() | 0xf0);
        check("vermicelliDoubleMaskedExec",
              vermicelliDoubleMaskedExec((char)(c1 & m1), (char)(c2 & m2), (char)m1, (char)m2,
                                         buf, end) - buf,
              orc_dverm_masked(c1 & m1, c2 & m2, m1, m2, buf, len), len);
        if (ds_ok) {
            check("shuftiDoubleExec",
                  shuftiDoubleExec(m128(dl1), m128(dh1), m128(dl2), m128(dh2), buf, end) - buf,
                  orc_shufti_double(dl1, dh1, dl2, dh2, buf, len, 64,
                                    (long)((uintptr_t)buf % 64)),
                  len);
        }
        /* run_accel over every scheme (AccelAux image, accel.h:72-146) */
        static const uint8_t types[] = {0, 1, 2, 3, 4, 13, 14, 15, 16, 17};
        for (size_t t = 0; t < sizeof(types); t++) {
            _Alignas(16) uint8_t aux[80];
            memset(aux, 0, sizeof(aux));
            aux[0] = types[t];
            aux[1] = (uint8_t)(rnd() % 4);
            if (types[t] == 13 && !sh_ok) continue;
            if (types[t] == 14 && !ds_ok) continue;
            switch (types[t]) {
            case 1: aux[2] = c1; break;
            case 2: aux[2] = uc1; break;
            case 3: aux[2] = c1; aux[3] = c2; break;
            case 4: aux[2] = uc1; aux[3] = (c2 >= 'a' && c2 <= 'z') ? c2 - 32 : c2; break;
            case 17: aux[2] = c1 & m1; aux[3] = c2 & m2; aux[4] = m1; aux[5] = m2; break;
            case 13: memcpy(aux + 16, lo, 16); memcpy(aux + 32, hi, 16); break;
            case 15: memcpy(aux + 16, t1, 16); memcpy(aux + 32, t2, 16); break;
            case 14:
                memcpy(aux + 16, dl1, 16); memcpy(aux + 32, dh1, 16);
                memcpy(aux + 48, dl2, 16); memcpy(aux + 64, dh2, 16);
                break;
            default: break;
            }
            char name[32];
            snprintf(name, sizeof name, "run_accel type %u", types[t]);
            check(name, run_accel((const union AccelAux *)aux, buf, end) - buf,
                  orc_run_accel(aux, buf, len), len);
        }
    }
    const int err = vsa_last_error();
    printf("abi_harness: %ld checks, %ld mismatches, last_error %d\n", checks, fails, err);
    free(raw);
    return (fails || err) ? 1 : 0;
}
