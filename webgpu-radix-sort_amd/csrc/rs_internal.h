// rs_internal.h — shared between librsort's translation units (not part of the C ABI).
#pragma once
#include "../../include/rsort.h"

// Sets the calling thread's rs_last_error() message (kept in rsort.hip) and returns s.
rs_status rs_internal_fail(rs_status s, const char* msg);

