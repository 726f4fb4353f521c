// ref_shim_avx.cpp -- extern "C" entry points onto the REFERENCE's AVX
// register kernels, which live inline in src/avxsort/avxsort_core.h (test
// infrastructure only: compiled with -mavx by oracle/build_ref.sh into
// oracle/_ref/libref8.so; tests/golden/make_golden.py pins the library's
// compat kernels with their outputs).
#include <stdint.h>

#include "avxsort_core.h"

extern "C" {

// avxsort_core.h:1213-1274 on nblocks consecutive blocks of 16 items
void ref_inregister_sort_keyval32(int64_t* items, int64_t* out, int64_t nblocks) {
    for (int64_t b = 0; b < nblocks; b++) inregister_sort_keyval32(items + 16 * b, out + 16 * b);
}

// avxsort_core.h:388-500: merge16_varlen writes the merged output AND flushes
// its last register into the consumed slots of one input (:461-475); the
// caller's copies of A and B come back as the kernel left them
void ref_merge16_varlen(int64_t* a, int64_t* b, int64_t* out, uint32_t la, uint32_t lb) {
    merge16_varlen(a, b, out, la, lb);
}

}  // extern "C"
