/*
 * hs_layout.h — the Vectorscan hot-path bytecode layouts, restated for the
 * MI355X engine.  Every struct here is byte-for-byte the reference layout so
 * that a blob produced by the reference compiler (or by our compile.cpp) is
 * consumed as-is; the static_asserts at the bottom pin the sizes/offsets the
 * survey measured (HWLM 176, noodTable 32, FDR 48, Teddy 24, FDRConfirm 32,
 * LitInfo 32, FDRFlood 208, AccelAux 80).
 *
 * Reference layouts:
 *   struct HWLM          src/hwlm/hwlm_internal.h:48-53   (engine at +ROUNDUP_CL)
 *   struct noodTable     src/hwlm/noodle_internal.h:38-47
 *   struct FDR           src/fdr/fdr_internal.h:69-85
 *   struct FDRFlood      src/fdr/fdr_internal.h:50-61
 *   struct Teddy         src/fdr/teddy_internal.h:56-63
 *   struct LitInfo       src/fdr/fdr_confirm.h:57-65
 *   struct FDRConfirm    src/fdr/fdr_confirm.h:78-83 (+ u32 litIndex[1<<nBits])
 *   union  AccelAux      src/nfa/accel.h:72-146
 */
#ifndef VSA_HS_LAYOUT_H
#define VSA_HS_LAYOUT_H

#include <stddef.h>
#include <stdint.h>

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64a;
typedef u64a hwlm_group_t;

#define VSA_CACHELINE 64
#define VSA_ROUNDUP_CL(x) (((x) + 63) & ~(size_t)63)
#define VSA_ROUNDUP_N(x, n) (((x) + (n)-1) & ~(size_t)((n)-1))

/* hwlm.h:59-75 */
#define HWLM_SUCCESS 0
#define HWLM_TERMINATED 1
#define HWLM_ERROR_UNKNOWN 2
#define HWLM_LITERAL_MAX_LEN 8
#define HWLM_ALL_GROUPS (~0ULL)
#define HWLM_CONTINUE_MATCHING HWLM_ALL_GROUPS
#define HWLM_TERMINATE_MATCHING 0ULL

/* hwlm_internal.h:38-41 */
#define HWLM_ENGINE_FDR 12
#define HWLM_ENGINE_NOOD 16

/* fdr_confirm.h:47, :67-68 */
#define FDR_LIT_FLAG_NOREPEAT 1
/* fdr_internal.h:48 */
#define FDR_FLOOD_MAX_IDS 16

/* accel.h:47-69 */
enum vsa_accel_type {
    ACCEL_NONE,
    ACCEL_VERM,
    ACCEL_VERM_NOCASE,
    ACCEL_DVERM,
    ACCEL_DVERM_NOCASE,
    ACCEL_RVERM,
    ACCEL_RVERM_NOCASE,
    ACCEL_RDVERM,
    ACCEL_RDVERM_NOCASE,
    ACCEL_REOD,
    ACCEL_REOD_NOCASE,
    ACCEL_RDEOD,
    ACCEL_RDEOD_NOCASE,
    ACCEL_SHUFTI,
    ACCEL_DSHUFTI,
    ACCEL_TRUFFLE,
    ACCEL_RED_TAPE,
    ACCEL_DVERM_MASKED,
    ACCEL_VERM16,
    ACCEL_DVERM16,
    ACCEL_DVERM16_MASKED,
};

typedef struct { u8 b[16]; } __attribute__((aligned(16))) vsa_m128;

/* accel.h:72 — only the members the HWLM header's accel schemes use. */
union AccelAux {
    u8 accel_type;
    struct { u8 accel_type; u8 offset; } generic;
    struct { u8 accel_type; u8 offset; u8 c; } verm;
    struct { u8 accel_type; u8 offset; u8 c1; u8 c2; u8 m1; u8 m2; } dverm;
    struct { u8 accel_type; u8 offset; vsa_m128 mask; } verm16;
    struct { u8 accel_type; u8 offset; vsa_m128 lo; vsa_m128 hi; } shufti;
    struct { u8 accel_type; u8 offset; vsa_m128 lo1; vsa_m128 hi1;
             vsa_m128 lo2; vsa_m128 hi2; } dshufti;
    struct { u8 accel_type; u8 offset; vsa_m128 mask1; vsa_m128 mask2; } truffle;
};

struct HWLM {
    u8 type;
    hwlm_group_t accel1_groups;
    union AccelAux accel1;
    union AccelAux accel0;
};

#define VSA_HWLM_C_DATA(p) \
    ((const void *)((const char *)(p) + VSA_ROUNDUP_CL(sizeof(struct HWLM))))

struct noodTable {
    u32 id;
    u64a msk;
    u64a cmp;
    u8 msk_len;
    u8 key_offset;
    u8 nocase;
    u8 single;
    u8 key0;
    u8 key1;
};

struct FDRFlood {
    hwlm_group_t allGroups;
    u32 suffix;
    u16 idCount;
    u32 ids[FDR_FLOOD_MAX_IDS];
    hwlm_group_t groups[FDR_FLOOD_MAX_IDS];
};

struct FDR {
    u32 engineID;
    u32 size;
    u32 maxStringLen;
    u32 numStrings;
    u32 confOffset;
    u32 floodOffset;
    u8 stride;
    u8 domain;
    u16 domainMask;
    u32 tabSize;
    vsa_m128 start;
};

struct Teddy {
    u32 engineID;
    u32 size;
    u32 maxStringLen;
    u32 numStrings;
    u32 confOffset;
    u32 floodOffset;
};

struct LitInfo {
    u64a v;
    u64a msk;
    hwlm_group_t groups;
    u32 id;
    u8 size;
    u8 flags;
    u8 next;
};

struct FDRConfirm {
    u64a andmsk;
    u64a mult;
    u32 nBits;
    hwlm_group_t groups;
};

/* Engine ids: fdr.c:776-796 funcs[] table; teddy_engine_description.cpp:52-69 */
#define VSA_ENGINE_FDR 0
#define VSA_TEDDY_FAT_FIRST 3
#define VSA_TEDDY_FAT_LAST 10
#define VSA_TEDDY_FIRST 11
#define VSA_TEDDY_LAST 18

static inline int vsa_engine_is_teddy(u32 id) {
    return id >= VSA_TEDDY_FAT_FIRST && id <= VSA_TEDDY_LAST;
}
static inline int vsa_engine_is_fat(u32 id) {
    return id >= VSA_TEDDY_FAT_FIRST && id <= VSA_TEDDY_FAT_LAST;
}
/* masks used by teddy engine id (1..4) */
static inline u32 vsa_teddy_num_masks(u32 id) {
    u32 base = vsa_engine_is_fat(id) ? VSA_TEDDY_FAT_FIRST : VSA_TEDDY_FIRST;
    return (id - base) / 2 + 1;
}

#ifdef __cplusplus
static_assert(sizeof(union AccelAux) == 80, "AccelAux layout");
static_assert(sizeof(struct HWLM) == 176, "HWLM layout");
static_assert(offsetof(struct HWLM, accel1) == 16, "HWLM.accel1");
static_assert(offsetof(struct HWLM, accel0) == 96, "HWLM.accel0");
static_assert(sizeof(struct noodTable) == 32, "noodTable layout");
static_assert(offsetof(struct noodTable, msk_len) == 24, "noodTable.msk_len");
static_assert(sizeof(struct FDR) == 48, "FDR layout");
static_assert(offsetof(struct FDR, start) == 32, "FDR.start");
static_assert(sizeof(struct Teddy) == 24, "Teddy layout");
static_assert(sizeof(struct LitInfo) == 32, "LitInfo layout");
static_assert(offsetof(struct LitInfo, next) == 30, "LitInfo.next");
static_assert(sizeof(struct FDRConfirm) == 32, "FDRConfirm layout");
static_assert(sizeof(struct FDRFlood) == 208, "FDRFlood layout");
#endif

#endif
