/*
 * compile.cpp — HWLM bytecode producer (noodle / FDR / Teddy / flood /
 * confirm) and accel mask builders.
 *
 * This is the "bytecode producer" row of SURVEY §2 (#3, #8, #10): it emits
 * blobs in exactly the reference layout (hs_layout.h) so the GPU engine and
 * the reference CPU runtime read the same bytes.  The algorithms follow the
 * reference compile side:
 *   literal normalisation     src/hwlm/hwlm_literal.cpp:85-117
 *   engine choice             src/hwlm/hwlm_build.cpp:164-214
 *   noodle table              src/hwlm/noodle_build.cpp:66-131
 *   FDR engine choice         src/fdr/fdr_engine_description.cpp:59-200
 *   FDR bucket assignment     src/fdr/fdr_compile.cpp:297-495
 *   FDR table                 src/fdr/fdr_compile.cpp:527-631
 *   FDR initial state         src/fdr/fdr_compile.cpp:129-151
 *   FDR layout                src/fdr/fdr_compile.cpp:159-211
 *   confirm tables            src/fdr/fdr_confirm_compile.cpp:75-336
 *   flood table               src/fdr/flood_compile.cpp:93-229
 *   Teddy engine choice       src/fdr/teddy_engine_description.cpp:52-200
 *   Teddy packing / masks     src/fdr/teddy_compile.cpp:138-618
 *   shufti / truffle masks    src/nfa/shufticompile.cpp:54-111,
 *                             src/nfa/trufflecompile.cpp:60-75
 * Not produced: Rose's included-literal squash masks (fdr_compile.cpp:
 * 640-805) live in the Rose program, not in the HWLM blob.
 */
#include "hs_layout.h"
#include "vsa_internal.h"

#include <algorithm>
#include <array>
#include <cassert>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <unordered_set>
#include <vector>

namespace vsa {

namespace {

static inline bool isUpper(u8 c) { return c >= 'A' && c <= 'Z'; }
static inline bool isLower(u8 c) { return c >= 'a' && c <= 'z'; }
static inline u8 toUpper(u8 c) { return isLower(c) ? c - 0x20 : c; }
static inline u8 toLower(u8 c) { return isUpper(c) ? c + 0x20 : c; }
static inline bool isAlpha(u8 c) { return toUpper(c) != toLower(c); }

static u32 lg2(u32 x) {
    u32 r = 0;
    while (x >>= 1) r++;
    return r;
}

static u32 absdiff(u32 a, u32 b) { return a > b ? a - b : b - a; }

/* ---------------------------------------------------------------- blobs */

struct Blob {
    u8 *p = nullptr;
    size_t size = 0;
    explicit Blob(size_t n) : size(n) {
        if (posix_memalign((void **)&p, 64, n ? n : 64)) {
            throw std::bad_alloc();
        }
        memset(p, 0, n ? n : 64);
    }
    Blob(const Blob &) = delete;
    Blob(Blob &&o) noexcept : p(o.p), size(o.size) { o.p = nullptr; o.size = 0; }
    Blob &operator=(Blob &&o) noexcept {
        if (this != &o) {
            free(p);
            p = o.p;
            size = o.size;
            o.p = nullptr;
            o.size = 0;
        }
        return *this;
    }
    ~Blob() { free(p); }
    u8 *release() { u8 *r = p; p = nullptr; return r; }
};

/* ------------------------------------------------------- flood control */

/* flood_compile.cpp:93-229 (FDRFlood per char, deduped, 256 x u32 index). */
static Blob buildFlood(const std::vector<Literal> &lits, u32 defaultSuffix,
                       bool allowFlood) {
    std::vector<FDRFlood> tmp(256);
    memset(tmp.data(), 0, sizeof(FDRFlood) * 256);
    for (auto &f : tmp) f.suffix = defaultSuffix;

    auto bumpSuffix = [&](u8 c, u32 suffix) {
        tmp[c].suffix = std::max(tmp[c].suffix, suffix + 1);
    };
    auto add = [&](u8 c, const Literal &lit, u32 suffix) {
        FDRFlood &fl = tmp[c];
        fl.suffix = std::max(fl.suffix, suffix + 1);
        if (fl.idCount < FDR_FLOOD_MAX_IDS) {
            fl.ids[fl.idCount] = lit.id;
            fl.allGroups |= lit.groups;
            fl.groups[fl.idCount] = lit.groups;
            fl.idCount++;
        }
    };

    for (const auto &lit : lits) {
        u32 litSize = (u32)lit.s.size();
        u32 maskSize = (u32)lit.msk.size();
        u8 c = (u8)lit.s[litSize - 1];
        bool nocase = isAlpha(c) ? lit.nocase : false;
        if (nocase && maskSize && (lit.msk[maskSize - 1] & 0x20)) {
            c = (lit.cmp[maskSize - 1] & 0x20) ? toLower(c) : toUpper(c);
            nocase = false;
        }
        u32 iEnd = std::max(litSize, maskSize);
        u32 up = iEnd, lo = iEnd;
        for (u32 i = 0; i < iEnd; i++) {
            if (i < litSize) {
                u8 d = (u8)lit.s[litSize - i - 1];
                bool diff = lit.nocase ? toLower(c) != toLower(d) : c != d;
                if (diff) {
                    up = std::min(up, i);
                    lo = std::min(lo, i);
                    break;
                }
            }
            if (i < maskSize) {
                u8 m = lit.msk[maskSize - i - 1];
                u8 cm = lit.cmp[maskSize - i - 1] & m;
                if (nocase) {
                    if ((toUpper(c) & m) != cm) up = std::min(up, i);
                    if ((toLower(c) & m) != cm) lo = std::min(lo, i);
                    if (lo != iEnd && up != iEnd) break;
                } else if ((c & m) != cm) {
                    up = std::min(up, i);
                    break;
                }
            }
        }
        u8 cu = nocase ? toUpper(c) : c;
        if (up != iEnd) bumpSuffix(cu, up); else add(cu, lit, up);
        if (nocase) {
            if (lo != iEnd) bumpSuffix(toLower(c), lo); else add(toLower(c), lit, lo);
        }
    }
    if (!allowFlood) {
        for (auto &f : tmp) f.idCount = FDR_FLOOD_MAX_IDS;
    }

    /* dedupe by raw bytes (FloodComparator is a memcmp order) */
    struct Cmp {
        bool operator()(const FDRFlood &a, const FDRFlood &b) const {
            return memcmp(&a, &b, sizeof(FDRFlood)) < 0;
        }
    };
    std::map<FDRFlood, std::vector<u32>, Cmp> distinct;
    for (u32 c = 0; c < 256; c++) distinct[tmp[c]].push_back(c);

    size_t hdr = sizeof(u32) * 256;
    size_t total = VSA_ROUNDUP_N(hdr + sizeof(FDRFlood) * distinct.size(), 16);
    Blob b(total);
    u32 *index = (u32 *)b.p;
    FDRFlood *recs = (FDRFlood *)(b.p + hdr);
    u32 k = 0;
    for (const auto &m : distinct) {
        memcpy(&recs[k], &m.first, sizeof(FDRFlood));
        for (u32 c : m.second) index[c] = k;
        k++;
    }
    return b;
}

/* ------------------------------------------------------------- confirm */

/* fdr_confirm_compile.cpp:52-66: bytes aligned to the top of the u64. */
static u64a topAlignedMask(const std::vector<u8> &v) {
    u64a m = 0;
    size_t n = std::min(v.size(), (size_t)8);
    memcpy((u8 *)&m + 8 - n, v.data() + v.size() - n, n);
    return m;
}

/* fdr_confirm_compile.cpp:75-129 */
static void litInfoFor(const Literal &lit, LitInfo &li) {
    memset(&li, 0, sizeof(li));
    li.id = lit.id;
    li.flags = lit.noruns ? FDR_LIT_FLAG_NOREPEAT : 0;
    li.size = (u8)std::max(lit.msk.size(), lit.s.size());
    li.groups = lit.groups;
    u64a msk = ~0ULL, val = 0;
    for (u32 j = 0; j < 8; j++) {
        u32 sh = (8 - j - 1) * 8;
        if (j >= lit.s.size()) {
            msk &= ~(0xffULL << sh);
        } else {
            u8 c = (u8)lit.s[lit.s.size() - j - 1];
            if (lit.nocase && isAlpha(c)) {
                msk &= ~(0x20ULL << sh);
                val |= (u64a)(c & 0xdf) << sh;
            } else {
                val |= (u64a)c << sh;
            }
        }
    }
    li.v = val;
    li.msk = msk;
    if (!lit.msk.empty()) {
        li.msk |= topAlignedMask(lit.msk);
        li.v |= topAlignedMask(lit.cmp);
    }
}

/* fdr_confirm_compile.cpp:132-254: one FDRConfirm + litIndex + LitInfo[] */
static Blob buildConfirm(const std::vector<Literal> &lits) {
    std::vector<LitInfo> info(lits.size());
    u64a andmsk = ~0ULL;
    for (size_t i = 0; i < lits.size(); i++) {
        litInfoFor(lits[i], info[i]);
        andmsk &= info[i].msk;
    }
    u32 nBits = lg2((u32)lits.size()) + 4;
    const u64a mult = 0x0b4e0ef37bc32127ULL;
    std::map<u32, std::vector<size_t>> byHash;
    hwlm_group_t gm = 0;
    for (size_t i = 0; i < lits.size(); i++) {
        u32 h = (u32)(((info[i].v & andmsk) * mult) >> (64 - nBits));
        byHash[h].push_back(i);
        gm |= info[i].groups;
    }
    size_t idxBytes = ((size_t)1 << nBits) * sizeof(u32);
    size_t size = VSA_ROUNDUP_N(sizeof(FDRConfirm), 4) +
                  VSA_ROUNDUP_N(idxBytes, 8) + sizeof(LitInfo) * lits.size();
    size = VSA_ROUNDUP_N(size, 8);
    Blob b(size);
    FDRConfirm *fc = (FDRConfirm *)b.p;
    fc->andmsk = andmsk;
    fc->mult = mult;
    fc->nBits = nBits;
    fc->groups = gm;
    u32 *litIndex = (u32 *)(b.p + VSA_ROUNDUP_N(sizeof(FDRConfirm), 4));
    u8 *ptr = (u8 *)litIndex + idxBytes;
    ptr = (u8 *)VSA_ROUNDUP_N((uintptr_t)ptr, 8);
    for (const auto &m : byHash) {
        litIndex[m.first] = (u32)(ptr - b.p);
        for (size_t k = 0; k < m.second.size(); k++) {
            LitInfo *li = (LitInfo *)ptr;
            *li = info[m.second[k]];
            li->next = (k + 1 == m.second.size()) ? 0 : 1;
            ptr += sizeof(LitInfo);
        }
    }
    size_t actual = VSA_ROUNDUP_N((size_t)(ptr - b.p), 8);
    b.size = actual;
    return b;
}

/* fdr_confirm_compile.cpp:293-336: confBase[nBuckets] (CL-rounded) then the
 * per-bucket confirm structures. */
static Blob buildFullConfirm(const std::vector<Literal> &lits,
                             const std::map<u32, std::vector<u32>> &b2l,
                             u32 nBuckets) {
    std::map<u32, Blob> per;
    size_t total = 0;
    for (u32 b = 0; b < nBuckets; b++) {
        auto it = b2l.find(b);
        if (it == b2l.end() || it->second.empty()) continue;
        std::vector<Literal> vl;
        for (u32 idx : it->second) vl.push_back(lits[idx]);
        Blob c = buildConfirm(vl);
        total += c.size;
        per.emplace(b, std::move(c));
    }
    size_t sw = VSA_ROUNDUP_CL(nBuckets * sizeof(u32));
    Blob out(sw + total);
    u32 *confBase = (u32 *)out.p;
    u8 *ptr = out.p + sw;
    for (auto &m : per) {
        confBase[m.first] = (u32)(ptr - out.p);
        memcpy(ptr, m.second.p, m.second.size);
        ptr += m.second.size;
    }
    return out;
}

/* ---------------------------------------------------------------- FDR */

struct FdrEngine {
    u32 bits = 0;
    u32 stride = 0;
};

/* fdr_engine_description.cpp:59-89 */
static u32 desiredStride(size_t numLits, size_t minLen, size_t minLenCount) {
    u32 d = 1;
    if (minLen > 1) {
        if (numLits < 250) d = (u32)minLen;
        else if (numLits < 800) d = (u32)minLen - 1;
        else if (numLits < 5000) d = (u32)std::min(minLen - 1, (size_t)2);
    }
    if (minLen == 4 && d == 4 && minLenCount > 2) d = 2;
    return d;
}

/* fdr_engine_description.cpp:91-200 (64-bit scheme, 8 buckets, not atom) */
static FdrEngine chooseFdr(const std::vector<Literal> &lits) {
    size_t msl = (size_t)-1, cnt = 0;
    for (auto &l : lits) {
        if (l.s.size() < msl) { msl = l.s.size(); cnt = 1; }
        else if (l.s.size() == msl) cnt++;
    }
    u32 want = desiredStride(lits.size(), msl, cnt);
    FdrEngine best;
    u32 bestScore = 0;
    bool have = false;
    for (u32 domain = 9; domain <= 15; domain++) {
        for (u32 stride = 1; stride <= 4; stride *= 2) {
            if (domain > 13 && stride > 1) continue;
            if (msl < stride) continue;
            u32 score = 100;
            score -= absdiff(want, stride);
            if (stride <= want) score += stride;
            u32 eff = (u32)lits.size();
            u32 ideal;
            if (eff < 8) ideal = stride == 1 ? 8 : 10;
            else if (eff < 20) ideal = 10;
            else if (eff < 100) ideal = 11;
            else if (eff < 1000) ideal = 12;
            else if (eff < 10000) ideal = 13;
            else ideal = 15;
            if (stride > 1) ideal++;
            score -= absdiff(ideal, domain);
            if (!have || score > bestScore) {
                best.bits = domain;
                best.stride = stride;
                bestScore = score;
                have = true;
            }
        }
    }
    return best;
}

/* fdr_compile.cpp:287-306 */
static bool nocaseCmpEq(const std::string &a, const std::string &b, bool nc) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); i++) {
        u8 x = (u8)a[i], y = (u8)b[i];
        if (nc) { x = toUpper(x); y = toUpper(y); }
        if (x != y) return false;
    }
    return true;
}

static bool isEquivLit(const Literal &a, const Literal &b, const Literal *lastNc) {
    if (a.s.size() != b.s.size()) return false;
    bool nc = lastNc && a.s.size() == lastNc->s.size() &&
              nocaseCmpEq(a.s, lastNc->s, true);
    return nocaseCmpEq(a.s, b.s, nc);
}

struct Chunk {
    u32 first_id, count, length;
};

/* fdr_compile.cpp:315-375 */
static std::vector<Chunk> assignChunks(const std::vector<Literal> &lits,
                                       size_t numLengths) {
    const u32 CHUNK_MAX = 512, MAX_CONSIDERED_LENGTH = 16;
    std::vector<Chunk> chunks;
    const u32 maxPerChunk = (u32)(lits.size() /
        (CHUNK_MAX - std::min((size_t)MAX_CONSIDERED_LENGTH, numLengths)) + 1);
    u32 curSize = 0, chunkStart = 0;
    const Literal *lastNc = nullptr;
    for (u32 i = 0; i < lits.size() && chunks.size() < CHUNK_MAX - 1; i++) {
        const auto &lit = lits[i];
        if (!(i != 0 && isEquivLit(lit, lits[i - 1], lastNc))) {
            if ((curSize < MAX_CONSIDERED_LENGTH && lit.s.size() != curSize) ||
                (curSize != 1 && (i - chunkStart) >= maxPerChunk)) {
                curSize = (u32)lit.s.size();
                if (!chunks.empty()) chunks.back().count = i - chunkStart;
                chunkStart = i;
                chunks.push_back({i, 0, curSize});
            }
        }
        if (lit.nocase) lastNc = &lit;
    }
    chunks.back().count = (u32)lits.size() - chunkStart;
    chunks.push_back({(u32)lits.size(), 0, 0});
    return chunks;
}

/* Scorer: pow(count, 1.05) * pow(len, -3), fdr_compile.cpp:223-285 */
static double score(u32 len, u32 count) {
    if (len == 0) return std::numeric_limits<double>::max();
    return std::pow((double)count, 1.05) * std::pow((double)len, -3.0);
}

/* fdr_compile.cpp:377-495; sorts lits in place */
static std::map<u32, std::vector<u32>> assignBuckets(std::vector<Literal> &lits,
                                                     u32 numBuckets) {
    std::map<u32, u32> lenCounts;
    for (auto &l : lits) lenCounts[(u32)l.s.size()]++;
    std::stable_sort(lits.begin(), lits.end(),
                     [](const Literal &a, const Literal &b) {
        if (a.s.size() != b.s.size()) return a.s.size() < b.s.size();
        auto p = std::mismatch(a.s.rbegin(), a.s.rend(), b.s.rbegin());
        if (p.first != a.s.rend()) return (char)*p.first < (char)*p.second;
        return a.nocase > b.nocase;
    });
    std::vector<Chunk> chunks = assignChunks(lits, lenCounts.size());
    const u32 nC = (u32)chunks.size();
    const double MAXS = std::numeric_limits<double>::max();
    std::vector<std::pair<double, u32>> t((size_t)nC * numBuckets);
    auto T = [&](u32 j, u32 i) -> std::pair<double, u32> & {
        return t[(size_t)j * numBuckets + i];
    };
    for (u32 j = 0; j < nC; j++) {
        u32 cnt = 0;
        for (u32 k = j; k < nC; k++) cnt += chunks[k].count;
        T(j, 0) = {score(chunks[j].length, cnt), 0};
    }
    for (u32 i = 1; i < numBuckets; i++) {
        for (u32 j = 0; j < nC - 1; j++) {
            std::pair<double, u32> best = {MAXS, 0};
            u32 cnt = chunks[j].count;
            for (u32 k = j + 1; k < nC - 1; k++) {
                double s = score(chunks[j].length, cnt);
                if (s > best.first) break;
                s += T(k, i - 1).first;
                if (s < best.first) best = {s, k};
                cnt += chunks[k].count;
            }
            T(j, i) = best;
        }
        T(nC - 1, i) = {0, 0};
    }
    std::vector<std::vector<u32>> buckets;
    for (u32 i = 0, n = numBuckets; n && i != nC - 1; n--) {
        u32 j = T(i, n - 1).second;
        if (j == 0) j = nC - 1;
        u32 first = chunks[i].first_id, last = chunks[j].first_id;
        std::vector<u32> ids;
        for (u32 k = 0; k < last - first; k++) ids.push_back(last - k - 1);
        i = j;
        buckets.push_back(ids);
    }
    std::map<u32, std::vector<u32>> b2l;
    for (size_t i = 0; i < buckets.size(); i++) {
        b2l.emplace((u32)(buckets.size() - i - 1), std::move(buckets[i]));
    }
    return b2l;
}

/* fdr_compile.cpp:527-570: (dontcare, value) of the domain key at `pos`;
 * returns true if the literal imposes no constraint there. */
static bool keyAtPosition(const Literal &lit, u32 bits, u32 pos, u32 *mask,
                          u32 *dc) {
    const u32 distance = bits <= 8 ? 1 : (bits <= 16 ? 2 : 4);
    const size_t sz = lit.s.size();
    u32 m = 0, d = 0;
    for (u32 cnt = 0; cnt < distance; cnt++) {
        int np = (int)pos - (int)cnt;
        u8 dcb = 0, mb = 0;
        if (np < 0 || (u32)np >= sz) {
            dcb = 0xff;
        } else {
            u8 c = (u8)lit.s[sz - np - 1];
            mb = c;
            u32 rem = bits - cnt * 8;
            if (rem < 8) {
                u8 cm = (u8)((1U << rem) - 1);
                mb &= cm;
                dcb |= (u8)~cm;
            }
            if (lit.nocase && isAlpha(c)) {
                mb &= 0xdf;
                dcb |= 0x20;
            }
        }
        m |= (u32)mb << (cnt * 8);
        d |= (u32)dcb << (cnt * 8);
    }
    u32 full = (1U << bits) - 1;
    m &= full;
    d &= full;
    *mask = m;
    *dc = d;
    return d == full;
}

/* fdr_compile.cpp:572-631 */
static std::vector<u64a> buildFdrTable(const std::vector<Literal> &lits,
                                       const std::map<u32, std::vector<u32>> &b2l,
                                       u32 bits) {
    const u32 n = 1U << bits;
    std::vector<u64a> tab(n, ~0ULL);
    u64a defaultMask = ~0ULL;
    for (u32 b = 0; b < 8; b++) {
        auto it = b2l.find(b);
        if (it == b2l.end()) continue;
        const auto &vl = it->second;
        for (u32 pos = 0; pos < 8; pos++) {
            u32 bit = pos * 8 + b;
            std::map<u32, std::unordered_set<u32>> m2;
            bool done = false;
            for (u32 idx : vl) {
                u32 m, dc;
                if (keyAtPosition(lits[idx], bits, pos, &m, &dc)) {
                    done = true;
                    break;
                }
                m2[dc].insert(m);
            }
            if (done) {
                defaultMask &= ~(1ULL << bit);
                continue;
            }
            for (const auto &e : m2) {
                u32 dc = e.first;
                /* enumerate all values of the don't-care bits */
                u32 v = ~dc;
                do {
                    u32 b2 = v & dc;
                    for (u32 mv : e.second) {
                        u32 val = (mv & ~dc) | b2;
                        tab[val] &= ~(1ULL << bit);
                    }
                    v = (v + (dc & (0U - dc))) | ~dc;
                } while (v != ~dc);
            }
        }
    }
    for (auto &x : tab) x &= defaultMask;
    return tab;
}

static Blob buildFdr(std::vector<Literal> lits, const BuildOptions &opt,
                     int hinted) {
    FdrEngine eng = chooseFdr(lits);
    if (hinted) {
        /* fdr_compile.cpp:862-866: hinted builds use domain 9, stride 1 */
        eng.bits = 9;
        eng.stride = 1;
    }
    auto b2l = assignBuckets(lits, 8);
    std::vector<u64a> tab = buildFdrTable(lits, b2l, eng.bits);
    /* default flood suffix: ((64 + 8 - 1) / 8) + 1 = 9
     * (fdr_engine_description.cpp:49-54) */
    Blob flood = buildFlood(lits, 9, opt.allow_flood);
    Blob conf = buildFullConfirm(lits, b2l, 8);

    size_t tabSize = tab.size() * 8;
    size_t size = VSA_ROUNDUP_CL(sizeof(FDR)) + VSA_ROUNDUP_CL(tabSize) +
                  VSA_ROUNDUP_CL(conf.size) + flood.size;
    Blob b(size);
    FDR *fdr = (FDR *)b.p;
    fdr->size = (u32)size;
    fdr->engineID = VSA_ENGINE_FDR;
    size_t maxLen = 0;
    for (auto &l : lits) maxLen = std::max(maxLen, l.s.size());
    fdr->maxStringLen = (u32)maxLen;
    fdr->numStrings = (u32)lits.size();
    fdr->domain = (u8)eng.bits;
    fdr->domainMask = (u16)((1U << eng.bits) - 1);
    fdr->tabSize = (u32)tabSize;
    fdr->stride = (u8)eng.stride;
    /* createInitialState: bit (pos, b) set for pos < minlen(b) - 1 */
    u8 *start = fdr->start.b;
    for (u32 bk = 0; bk < 8; bk++) {
        auto it = b2l.find(bk);
        u32 minLen = ~0U;
        if (it != b2l.end()) {
            for (u32 idx : it->second) minLen = std::min(minLen, (u32)lits[idx].s.size());
        }
        for (u32 i = 0; i < 8; i++) {
            if (i + 1 < minLen) {
                u32 bit = i * 8 + bk;
                start[bit / 8] |= (u8)(1U << (bit % 8));
            }
        }
    }
    u8 *ptr = b.p + VSA_ROUNDUP_CL(sizeof(FDR));
    memcpy(ptr, tab.data(), tabSize);
    ptr += VSA_ROUNDUP_CL(tabSize);
    fdr->confOffset = (u32)(ptr - b.p);
    memcpy(ptr, conf.p, conf.size);
    ptr += VSA_ROUNDUP_CL(conf.size);
    fdr->floodOffset = (u32)(ptr - b.p);
    memcpy(ptr, flood.p, flood.size);
    return b;
}

/* --------------------------------------------------------------- Teddy */

struct TeddyDef {
    u32 id, numMasks, numBuckets;
    bool packed, fat;
};

static const TeddyDef kTeddyDefs[] = {
    {3, 1, 16, false, true},  {4, 1, 16, true, true},
    {5, 2, 16, false, true},  {6, 2, 16, true, true},
    {7, 3, 16, false, true},  {8, 3, 16, true, true},
    {9, 4, 16, false, true},  {10, 4, 16, true, true},
    {11, 1, 8, false, false}, {12, 1, 8, true, false},
    {13, 2, 8, false, false}, {14, 2, 8, true, false},
    {15, 3, 8, false, false}, {16, 3, 8, true, false},
    {17, 4, 8, false, false}, {18, 4, 8, true, false},
};

static const u32 TEDDY_BUCKET_LOAD = 6;

/* teddy_engine_description.cpp:76-124 */
static bool teddyAllowed(const std::vector<Literal> &vl, const TeddyDef &e,
                         size_t maxLen, bool allowFat) {
    if (e.fat && !allowFat) return false;
    if (e.numBuckets < vl.size() && !e.packed) return false;
    if (e.numBuckets * TEDDY_BUCKET_LOAD < vl.size()) return false;
    if (e.numMasks > maxLen) return false;
    if (vl.size() > 40) {
        u32 nSmall = 0;
        for (auto &l : vl) if (l.s.size() < e.numMasks) nSmall++;
        if (nSmall * 5 > vl.size()) return false;
    }
    return true;
}

/* teddy_engine_description.cpp:126-188 */
static const TeddyDef *chooseTeddy(const std::vector<Literal> &vl, bool allowFat) {
    size_t maxLen = 0, maxFloodTail = 0;
    for (auto &l : vl) {
        maxLen = std::max(maxLen, l.s.size());
        size_t j;
        for (j = 1; j < l.s.size(); j++) {
            if (l.s[l.s.size() - j - 1] != l.s[l.s.size() - 1]) break;
        }
        maxFloodTail = std::max(maxFloodTail, j);
    }
    const TeddyDef *best = nullptr;
    u32 bestScore = 0;
    for (const auto &e : kTeddyDefs) {
        if (!teddyAllowed(vl, e, maxLen, allowFat)) continue;
        u32 s = 0;
        if (!e.packed) s += 100;
        if (vl.size() > 4 * e.numBuckets) s += e.numMasks * 4;
        else s += 100;
        if (e.numMasks > maxFloodTail) s += 50;
        s += 6 / (std::abs(3 - (int)e.numMasks) + 1);
        s += 16 / e.numBuckets;
        if (!best || s > bestScore) { best = &e; bestScore = s; }
    }
    return best;
}

/* TeddySet: teddy_compile.cpp:94-221 */
struct TeddySet {
    u32 len;
    std::vector<u16> nib;
    std::vector<u32> ids;
    explicit TeddySet(u32 l) : len(l), nib(l * 2, 0) {}
    bool operator<(const TeddySet &o) const { return ids < o.ids; }
    void add(u32 id, const Literal &lit) {
        const std::string &s = lit.s;
        for (u32 i = 0; i < len; i++) {
            if (i < s.size()) {
                u8 c = (u8)s[s.size() - i - 1];
                u8 hi = (c >> 4) & 0xf, lo = c & 0xf;
                nib[i * 2] = (u16)(1U << lo);
                if (lit.nocase && isAlpha(c)) {
                    nib[i * 2 + 1] = (u16)((1U << (hi & 0xd)) | (1U << (hi | 0x2)));
                } else {
                    nib[i * 2 + 1] = (u16)(1U << hi);
                }
            } else {
                nib[i * 2] = nib[i * 2 + 1] = 0xffff;
            }
        }
        ids.push_back(id);
        std::sort(ids.begin(), ids.end());
        ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    }
    u64a probability() const {
        u64a v = 1;
        for (u16 x : nib) v *= (u64a)__builtin_popcount(x);
        return v;
    }
    u64a heuristic() const { return probability() * (2 + ids.size()); }
    bool runProne() const {
        u16 la = 0xffff, ha = 0xffff;
        for (u32 i = 0; i < len; i++) { la &= nib[i * 2]; ha &= nib[i * 2 + 1]; }
        return la && ha;
    }
    bool identicalTail(const TeddySet &o) const { return nib == o.nib; }
};

static TeddySet mergeSets(const TeddySet &a, const TeddySet &b) {
    TeddySet m(a);
    for (size_t i = 0; i < m.nib.size(); i++) m.nib[i] |= b.nib[i];
    m.ids.insert(m.ids.end(), b.ids.begin(), b.ids.end());
    std::sort(m.ids.begin(), m.ids.end());
    m.ids.erase(std::unique(m.ids.begin(), m.ids.end()), m.ids.end());
    return m;
}

/* teddy_compile.cpp:223-318 */
static bool teddyPack(const std::vector<Literal> &lits, const TeddyDef &e,
                      std::map<u32, std::vector<u32>> &b2l) {
    std::set<TeddySet> sts;
    for (u32 i = 0; i < lits.size(); i++) {
        TeddySet ts(e.numMasks);
        ts.add(i, lits[i]);
        sts.insert(ts);
    }
    while (true) {
        auto m1 = sts.end(), m2 = sts.end();
        u64a best = ~0ULL;
        for (auto i1 = sts.begin(); i1 != sts.end(); ++i1) {
            auto i2 = i1;
            for (++i2; i2 != sts.end(); ++i2) {
                if (sts.size() <= e.numBuckets && !i1->identicalTail(*i2)) continue;
                TeddySet tmp = mergeSets(*i1, *i2);
                u64a ns = tmp.heuristic();
                u64a os = i1->heuristic() + i2->heuristic();
                if (ns < os) {
                    /* the reference breaks the inner loop only; later outer
                     * iterations may still replace the choice */
                    m1 = i1;
                    m2 = i2;
                    break;
                }
                u64a sc = ns - os;
                bool oldRun = i1->runProne() && i2->runProne();
                if (tmp.runProne() && !oldRun) continue;
                if (sc < best) { best = sc; m1 = i1; m2 = i2; }
            }
        }
        if (m1 == sts.end() || m2 == sts.end()) break;
        TeddySet nts = mergeSets(*m1, *m2);
        sts.erase(m1);
        sts.erase(m2);
        sts.insert(nts);
    }
    if (sts.size() > e.numBuckets) return false;
    u32 bid = 0;
    for (const auto &ts : sts) {
        auto &bl = b2l[bid++];
        bl.insert(bl.end(), ts.ids.begin(), ts.ids.end());
    }
    return true;
}

/* fillNibbleMasks, teddy_compile.cpp:439-509 (maskWidth 1 or 2) */
static void fillNibbleMasks(const std::map<u32, std::vector<u32>> &b2l,
                            const std::vector<Literal> &lits, u32 numMasks,
                            u32 maskWidth, u32 chunk, u8 *base, size_t len,
                            bool dupLayout) {
    memset(base, 0xff, len);
    for (const auto &e : b2l) {
        u32 bid = e.first;
        u8 bmsk = (u8)(1U << (bid % 8));
        for (u32 li : e.second) {
            const Literal &l = lits[li];
            u32 sz = (u32)l.s.size();
            for (u32 j = 0; j < numMasks; j++) {
                u32 idLo = j * 2 * maskWidth + bid / 8;
                u32 idHi = (j * 2 + 1) * maskWidth + bid / 8;
                /* dup layout (fat teddy copy): each 16-B mask stored twice */
                u32 copies = dupLayout ? 2 : 1;
                for (u32 cp = 0; cp < copies; cp++) {
                    u32 loBase = idLo * chunk + cp * 16;
                    u32 hiBase = idHi * chunk + cp * 16;
                    if (j >= sz) {
                        for (u32 n = 0; n < 16; n++) {
                            base[loBase + n] &= ~bmsk;
                            base[hiBase + n] &= ~bmsk;
                        }
                        continue;
                    }
                    u8 c = (u8)l.s[sz - 1 - j];
                    u32 nHi = (c >> 4) & 0xf, nLo = c & 0xf;
                    if (j < l.msk.size() && l.msk[l.msk.size() - 1 - j]) {
                        u8 m = l.msk[l.msk.size() - 1 - j];
                        u8 cmpv = l.cmp[l.msk.size() - 1 - j];
                        u8 mLo = m & 0xf, mHi = (m >> 4) & 0xf;
                        u8 cLo = cmpv & 0xf, cHi = (cmpv >> 4) & 0xf;
                        for (u8 cm = 0; cm < 16; cm++) {
                            if ((cm & mLo) == (cLo & mLo)) base[loBase + cm] &= ~bmsk;
                            if ((cm & mHi) == (cHi & mHi)) base[hiBase + cm] &= ~bmsk;
                        }
                    } else {
                        if (l.nocase && isAlpha(c)) {
                            base[hiBase + (nHi & 0xd)] &= ~bmsk;
                            base[hiBase + (nHi | 0x2)] &= ~bmsk;
                        } else {
                            base[hiBase + nHi] &= ~bmsk;
                        }
                        base[loBase + nLo] &= ~bmsk;
                    }
                }
            }
        }
    }
}

/* fillReinforcedTable, teddy_compile.cpp:511-552 (8-bucket Teddy only) */
static void fillReinforced(const std::map<u32, std::vector<u32>> &b2l,
                           const std::vector<Literal> &lits, u8 *rt) {
    u64a *m = (u64a *)rt;
    for (u32 i = 0; i < 256; i++) m[i] = 0x00ffffffffffffffULL;
    auto clr = [&](int c, u32 j, u8 bm) {
        if (c < 0) {
            for (u32 i = 0; i < 256; i++) rt[i * 8 + j - 1] &= ~bm;
        } else {
            rt[c * 8 + j - 1] &= ~bm;
        }
    };
    for (const auto &e : b2l) {
        u8 bm = (u8)(1U << (e.first % 8));
        for (u32 li : e.second) {
            const Literal &l = lits[li];
            u32 sz = (u32)l.s.size();
            for (u32 j = 1; j < 8; j++) {
                if (sz - 1 < j) {
                    clr(-1, j, bm);
                } else {
                    u8 c = (u8)l.s[sz - 1 - j];
                    if (l.nocase && isAlpha(c)) {
                        clr(c & 0xdf, j, bm);
                        clr(c | 0x20, j, bm);
                    } else {
                        clr(c, j, bm);
                    }
                }
            }
        }
    }
    memset(rt + 256 * 8, 0, 8);
}

static Blob buildTeddy(const std::vector<Literal> &lits, const TeddyDef &e,
                       const std::map<u32, std::vector<u32>> &b2l,
                       const BuildOptions &opt) {
    u32 maskWidth = e.numBuckets / 8;
    size_t maskLen = (size_t)e.numMasks * 16 * 2 * maskWidth;
    size_t rLen = (size_t)(256 + 1) * 8 * maskWidth;
    if (maskWidth == 2) rLen = maskLen * 2;
    Blob flood = buildFlood(lits, e.numMasks, opt.allow_flood);
    Blob conf = buildFullConfirm(lits, b2l, e.numBuckets);
    size_t size = VSA_ROUNDUP_CL(sizeof(Teddy)) + VSA_ROUNDUP_CL(maskLen) +
                  VSA_ROUNDUP_CL(rLen) + VSA_ROUNDUP_CL(conf.size) + flood.size;
    Blob b(size);
    Teddy *t = (Teddy *)b.p;
    t->size = (u32)size;
    t->engineID = e.id;
    size_t maxLen = 0;
    for (auto &l : lits) maxLen = std::max(maxLen, l.s.size());
    t->maxStringLen = (u32)maxLen;
    t->numStrings = (u32)lits.size();
    u8 *ptr = b.p + VSA_ROUNDUP_CL(sizeof(Teddy)) + VSA_ROUNDUP_CL(maskLen) +
              VSA_ROUNDUP_CL(rLen);
    t->confOffset = (u32)(ptr - b.p);
    memcpy(ptr, conf.p, conf.size);
    ptr += VSA_ROUNDUP_CL(conf.size);
    t->floodOffset = (u32)(ptr - b.p);
    memcpy(ptr, flood.p, flood.size);
    u8 *baseMsk = b.p + VSA_ROUNDUP_CL(sizeof(Teddy));
    fillNibbleMasks(b2l, lits, e.numMasks, maskWidth, 16, baseMsk, maskLen, false);
    if (maskWidth == 1) {
        fillReinforced(b2l, lits, baseMsk + VSA_ROUNDUP_CL(maskLen));
    } else {
        /* fillDupNibbleMasks: same masks, 32-B stride, each half duplicated */
        fillNibbleMasks(b2l, lits, e.numMasks, maskWidth, 32,
                        baseMsk + VSA_ROUNDUP_CL(maskLen), rLen, true);
    }
    return b;
}

/* --------------------------------------------------------------- noodle */

/* noodle_build.cpp:66-131 */
static Blob buildNoodle(const Literal &lit) {
    const std::string &s = lit.s;
    size_t maskLen = std::max(s.size(), lit.msk.size());
    std::vector<u8> nm(maskLen, 0), nc(maskLen, 0);
    for (size_t i = maskLen - lit.msk.size(), j = 0; i < maskLen; i++, j++) {
        nm[i] = lit.msk[j];
        nc[i] = lit.cmp[j];
    }
    size_t off = maskLen - s.size();
    for (size_t i = off; i < maskLen; i++) {
        u8 c = (u8)s[i - off];
        u8 sm = lit.nocase && isAlpha(c) ? 0xdf : 0xff;
        nm[i] |= sm;
        nc[i] |= c & sm;
    }
    size_t keyOff = 0;
    for (size_t i = 0; i + 1 < s.size(); i++) {
        u8 c = (u8)s[i], d = (u8)s[i + 1];
        bool diff = (lit.nocase && isAlpha(c)) ? toUpper(c) != toUpper(d) : c != d;
        keyOff = i;
        if (diff) break;
    }
    Blob b(sizeof(noodTable));
    noodTable *n = (noodTable *)b.p;
    n->id = lit.id;
    n->single = s.size() == 1 ? 1 : 0;
    n->key_offset = (u8)(s.size() - keyOff);
    n->nocase = lit.nocase ? 1 : 0;
    n->key0 = (u8)s[keyOff];
    n->key1 = n->single ? 0 : (u8)s[keyOff + 1];
    memcpy(&n->msk, nm.data(), maskLen);
    memcpy(&n->cmp, nc.data(), maskLen);
    n->msk_len = (u8)maskLen;
    return b;
}

} // namespace

/* hwlm_literal.cpp:85-117 */
Literal makeLiteral(const u8 *s, size_t len, bool nocase, bool noruns, u32 id,
                    u64a groups, const u8 *msk, const u8 *cmp, size_t mlen) {
    Literal l;
    l.s.assign((const char *)s, len);
    l.nocase = nocase;
    l.noruns = noruns;
    l.id = id;
    l.groups = groups;
    if (mlen) {
        l.msk.assign(msk, msk + mlen);
        l.cmp.assign(cmp, cmp + mlen);
    }
    if (nocase) {
        for (auto &c : l.s) c = (char)toUpper((u8)c);
    }
    bool allZero = std::all_of(l.msk.begin(), l.msk.end(), [](u8 v) { return v == 0; });
    if (allZero) {
        l.msk.clear();
        l.cmp.clear();
    }
    return l;
}

/* hwlm_build.cpp:120-214 plus fdr_compile.cpp:837-897 */
int buildHwlm(std::vector<Literal> lits, const BuildOptions &opt, u8 **out,
              size_t *outSize) {
    if (lits.empty()) return VSA_E_INVALID;
    for (auto &l : lits) {
        if (l.s.empty() || l.s.size() > HWLM_LITERAL_MAX_LEN ||
            l.msk.size() > 8 || l.msk.size() != l.cmp.size() ||
            l.id == 0xffffffffu || !l.groups) {
            return VSA_E_INVALID;
        }
    }
    try {
        u8 type;
        Blob eng(0);
        int hint = opt.engine_hint;
        if (lits.size() == 1 && opt.allow_noodle && hint < 0) {
            type = HWLM_ENGINE_NOOD;
            eng = buildNoodle(lits[0]);
        } else {
            type = HWLM_ENGINE_FDR;
            bool built = false;
            if (opt.allow_teddy && (hint < 0 || hint >= (int)VSA_TEDDY_FAT_FIRST)) {
                const TeddyDef *td = nullptr;
                if (hint < 0) {
                    td = chooseTeddy(lits, opt.allow_fat_teddy);
                } else {
                    for (const auto &d : kTeddyDefs) if ((int)d.id == hint) td = &d;
                }
                if (td) {
                    std::map<u32, std::vector<u32>> b2l;
                    if (lits.size() <= td->numBuckets * TEDDY_BUCKET_LOAD &&
                        teddyPack(lits, *td, b2l)) {
                        eng = buildTeddy(lits, *td, b2l, opt);
                        built = true;
                    }
                }
                if (!built && hint >= 0) return VSA_E_NOT_BUILDABLE;
            }
            if (!built) {
                if (hint > 0) return VSA_E_NOT_BUILDABLE;
                eng = buildFdr(lits, opt, hint == 0);
            }
        }
        size_t total = VSA_ROUNDUP_CL(sizeof(HWLM)) + eng.size;
        Blob h(total);
        HWLM *hw = (HWLM *)h.p;
        hw->type = type;
        memcpy(h.p + VSA_ROUNDUP_CL(sizeof(HWLM)), eng.p, eng.size);
        *outSize = total;
        *out = h.release();
        return VSA_OK;
    } catch (const std::bad_alloc &) {
        return VSA_E_NOMEM;
    }
}

/* shufticompile.cpp:54-111: class -> (lo, hi) nibble masks, or -1. */
int shuftiMasks(const u8 cls[32], u8 lo[16], u8 hi[16]) {
    std::map<u8, u16> byHi;
    for (u32 c = 0; c < 256; c++) {
        if (cls[c >> 3] & (1U << (c & 7))) byHi[(u8)(c >> 4)] |= (u16)(1U << (c & 15));
    }
    std::map<u16, u16> byLoSet;
    for (auto &e : byHi) byLoSet[e.second] |= (u16)(1U << e.first);
    if (byLoSet.size() > 8) return -1;
    memset(lo, 0, 16);
    memset(hi, 0, 16);
    u32 bit = 0;
    for (auto &e : byLoSet) {
        for (u32 j = 0; j < 16; j++) {
            if (e.first & (1U << j)) lo[j] |= (u8)(1U << bit);
            if (e.second & (1U << j)) hi[j] |= (u8)(1U << bit);
        }
        bit++;
    }
    return (int)bit;
}

/* shufticompile.cpp:135-209 (shuftiBuildDoubleMasks): one-byte literals
 * (second byte wildcard) and two-byte literals -> bucketed nibble masks,
 * bit clear = member.  Literals sharing three of their four nibble sets are
 * merged (four passes, std::map order), at most 8 buckets; false = too many.
 * pairs: npairs (first, second) byte pairs in flat_set (sorted) order. */
bool shuftiDoubleMasks(const u8 onechar[32], const u8 *pairs, size_t npairs, u8 lo1[16],
                       u8 hi1[16], u8 lo2[16], u8 hi2[16]) {
    typedef std::array<u16, 4> NM;
    std::vector<std::pair<u8, u8>> tw;
    for (size_t i = 0; i < npairs; i++) tw.emplace_back(pairs[2 * i], pairs[2 * i + 1]);
    std::sort(tw.begin(), tw.end());
    tw.erase(std::unique(tw.begin(), tw.end()), tw.end());
    std::vector<NM> nm;
    for (auto &p : tw) {
        nm.push_back({{(u16)(1U << (p.first & 0xf)), (u16)(1U << (p.first >> 4)),
                       (u16)(1U << (p.second & 0xf)), (u16)(1U << (p.second >> 4))}});
    }
    for (u32 c = 0; c < 256; c++) {
        if (onechar && (onechar[c >> 3] & (1U << (c & 7)))) {
            nm.push_back({{(u16)(1U << (c & 0xf)), (u16)(1U << (c >> 4)), 0xffff, 0xffff}});
        }
    }
    for (u32 i = 0; i < 4; i++) {
        std::map<NM, NM> merged;
        for (const auto &a : nm) {
            NM key = a;
            key[i] = 0;
            auto it = merged.find(key);
            if (it == merged.end()) {
                merged[key] = a;
            } else {
                for (int k = 0; k < 4; k++) it->second[k] |= a[k];
            }
        }
        nm.clear();
        for (auto &e : merged) nm.push_back(e.second);
    }
    if (nm.size() > 8) return false;
    u8 *out[4] = {lo1, hi1, lo2, hi2};
    for (int k = 0; k < 4; k++) memset(out[k], 0xff, 16);
    u32 bucket = 0;
    for (const auto &a : nm) {
        for (int k = 0; k < 4; k++) {
            for (u32 n = 0; n < 16; n++) {
                if (a[k] & (1U << n)) out[k][n] &= (u8)~(1U << bucket);
            }
        }
        bucket++;
    }
    return true;
}

/* trufflecompile.cpp:60-75 */
void truffleMasks(const u8 cls[32], u8 m1[16], u8 m2[16]) {
    memset(m1, 0, 16);
    memset(m2, 0, 16);
    for (u32 v = 0; v < 256; v++) {
        if (!(cls[v >> 3] & (1U << (v & 7)))) continue;
        u8 *m = (v & 0x80) ? m2 : m1;
        m[v & 0xf] |= (u8)(1U << ((v & 0x70) >> 4));
    }
}

} // namespace vsa
