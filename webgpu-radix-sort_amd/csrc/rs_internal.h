// rs_internal.h — shared between librsort's translation units (not part of the C ABI).
#pragma once
#include "../../include/rsort.h"

// Sets the calling thread's rs_last_error() message (kept in rsort.hip) and returns s.
rs_status rs_internal_fail(rs_status s, const char* msg);

// Out-of-place whole sort (multi-GPU group at world size 1): in[0..n) only read, the result in
// out[0..n); a plan with separate values or keys only, no check_order.
rs_status rs_internal_sort_from(rs_plan* p, const void* in_k, const void* in_v, void* out_k,
                                void* out_v, uint64_t n, void* stream);
