// ldpc_internal.h -- shared helpers of libldpc_hip.so (not part of the ABI).
#pragma once
#include <cstdarg>
#include <cstdio>

#include "../../include/ldpc_hip.h"

// Records a thread-local message for ldpc_last_error() and returns `code`.
int ldpc_fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
