/*
 * vectorscan_amd_hs_names.h — the reference's hs-layer names over the
 * pure-literal database API (vectorscan_amd_hs.h), for a program written
 * against <hs.h> whose databases hold only pure literals
 * (hs_compile_lit / hs_compile_lit_multi): include this header instead of
 * <hs.h> and link libvectorscan_amd.so; the calls, types, flags and return
 * codes keep their reference names (hs_common.h, hs_compile.h,
 * hs_runtime.h).  Source-level only: the library exports the vsa_hs_*
 * symbols, so a program can also link the reference's libhs beside it.
 * hs_compile / hs_compile_multi (regular expressions) and the rest of the
 * reference's API are not provided.  tests/c/hs_names_demo.c is such a
 * program, checked against a brute-force scan of its own buffer.
 */
#ifndef VECTORSCAN_AMD_HS_NAMES_H
#define VECTORSCAN_AMD_HS_NAMES_H

#if defined(HS_H_) || defined(HS_COMMON_H_) || defined(HS_RUNTIME_H_) || defined(HS_COMPILE_H_)
#error "vectorscan_amd_hs_names.h replaces <hs.h>: include one or the other"
#endif

#include "vectorscan_amd_hs.h"

/* hs_common.h:478-584 */
#define HS_SUCCESS VSA_HS_SUCCESS
#define HS_INVALID VSA_HS_INVALID
#define HS_NOMEM VSA_HS_NOMEM
#define HS_SCAN_TERMINATED VSA_HS_SCAN_TERMINATED
#define HS_COMPILER_ERROR VSA_HS_COMPILER_ERROR
#define HS_DB_VERSION_ERROR VSA_HS_DB_VERSION_ERROR
#define HS_DB_PLATFORM_ERROR VSA_HS_DB_PLATFORM_ERROR
#define HS_DB_MODE_ERROR VSA_HS_DB_MODE_ERROR
#define HS_SCRATCH_IN_USE VSA_HS_SCRATCH_IN_USE
#define HS_UNKNOWN_ERROR VSA_HS_UNKNOWN_ERROR

/* hs_compile.h:869-1005, 1156-1171 */
#define HS_FLAG_CASELESS VSA_HS_FLAG_CASELESS
#define HS_FLAG_DOTALL VSA_HS_FLAG_DOTALL
#define HS_FLAG_MULTILINE VSA_HS_FLAG_MULTILINE
#define HS_FLAG_SINGLEMATCH VSA_HS_FLAG_SINGLEMATCH
#define HS_FLAG_ALLOWEMPTY VSA_HS_FLAG_ALLOWEMPTY
#define HS_FLAG_UTF8 VSA_HS_FLAG_UTF8
#define HS_FLAG_UCP VSA_HS_FLAG_UCP
#define HS_FLAG_PREFILTER VSA_HS_FLAG_PREFILTER
#define HS_FLAG_SOM_LEFTMOST VSA_HS_FLAG_SOM_LEFTMOST
#define HS_FLAG_COMBINATION VSA_HS_FLAG_COMBINATION
#define HS_FLAG_QUIET VSA_HS_FLAG_QUIET
#define HS_MODE_BLOCK VSA_HS_MODE_BLOCK
#define HS_MODE_NOSTREAM VSA_HS_MODE_BLOCK
#define HS_MODE_STREAM VSA_HS_MODE_STREAM
#define HS_MODE_VECTORED VSA_HS_MODE_VECTORED
#define HS_MODE_SOM_HORIZON_LARGE VSA_HS_MODE_SOM_HORIZON_LARGE
#define HS_MODE_SOM_HORIZON_MEDIUM VSA_HS_MODE_SOM_HORIZON_MEDIUM
#define HS_MODE_SOM_HORIZON_SMALL VSA_HS_MODE_SOM_HORIZON_SMALL

/* hs_common.h:80-104, hs_compile.h:112-130, hs_runtime.h:63-128 */
typedef vsa_hs_database_t hs_database_t;
typedef vsa_hs_scratch_t hs_scratch_t;
typedef vsa_hs_stream_t hs_stream_t;
typedef vsa_hs_compile_error_t hs_compile_error_t;
typedef vsa_hs_match_event_handler match_event_handler;
typedef int hs_error_t;

/* the calls (the header beside each vsa_hs_* declaration cites the
 * reference's) */
#define hs_compile_lit vsa_hs_compile_lit
#define hs_compile_lit_multi vsa_hs_compile_lit_multi
#define hs_free_compile_error vsa_hs_free_compile_error
#define hs_free_database vsa_hs_free_database
#define hs_alloc_scratch vsa_hs_alloc_scratch
#define hs_free_scratch vsa_hs_free_scratch
#define hs_clone_scratch vsa_hs_clone_scratch
#define hs_scratch_size vsa_hs_scratch_size
#define hs_scan vsa_hs_scan
#define hs_scan_vector vsa_hs_scan_vector
#define hs_open_stream vsa_hs_open_stream
#define hs_scan_stream vsa_hs_scan_stream
#define hs_close_stream vsa_hs_close_stream
#define hs_reset_stream vsa_hs_reset_stream
#define hs_copy_stream vsa_hs_copy_stream
#define hs_reset_and_copy_stream vsa_hs_reset_and_copy_stream
#define hs_stream_size vsa_hs_stream_size
#define hs_serialize_database vsa_hs_serialize_database
#define hs_deserialize_database vsa_hs_deserialize_database
#define hs_serialized_database_size vsa_hs_serialized_database_size
#define hs_serialized_database_info vsa_hs_serialized_database_info
#define hs_database_size vsa_hs_database_size
#define hs_database_info vsa_hs_database_info
#define hs_valid_platform vsa_hs_valid_platform
#define hs_version vsa_hs_version

#endif
