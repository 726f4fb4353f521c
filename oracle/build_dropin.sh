#!/usr/bin/env bash
# Drop-in check: the reference's own drivers and check_* tests, compiled from
# their sources where they lie in /root/reference, against the reference-named
# headers in include/compat/ and linked with the MI355X library instead of the
# AVX objects.  Outputs only into oracle/_ref/dropin/
# (git-ignored, shipped to the GPU box with the tree); tests/test_dropin.py
# runs them there.  check.h is the minimal harness in tests/compat_check/.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
ROOT="$(dirname "$HERE")"
REF="${SMJ_REFERENCE:-/root/reference}"
S="$REF/src"
T="$REF/tests"
if [ ! -d "$S" ]; then
    echo "[build_dropin] $REF not present: drop-in binaries not rebuilt"
    exit 0
fi
OUT="$HERE/_ref/dropin"
LIB="$ROOT/avx-sort-merge-joins_amd/lib"
mkdir -p "$OUT"
CC="${CC:-gcc}"
CXX="${CXX:-g++}"
INC="-I$ROOT/include/compat -I$ROOT/tests/compat_check -I$REF -I$S -I$S/util -I$S/datagen -I$T"
FLAGS="-O2 -std=gnu99 -D_GNU_SOURCE -w"
RPATH='-Wl,-rpath,$ORIGIN/../../../avx-sort-merge-joins_amd/lib'
GEN="$S/datagen/generator.c $S/datagen/genzipf.c $S/util/cpu_mapping.c"
build() {  # name width sources...
    local name=$1 w=$2; shift 2
    local def="" lib="-lsmj_hip"
    if [ "$w" = 16 ]; then def="-DKEY_8B"; lib="-lsmj_hip_k8"; fi
    $CC $FLAGS $def $INC "$@" -L"$LIB" $lib $RPATH -lpthread -lm -o "$OUT/$name$w"
}
buildxx() {  # C++ drivers (sortbench.c includes <algorithm>)
    local name=$1 w=$2; shift 2
    local def="" lib="-lsmj_hip"
    if [ "$w" = 16 ]; then def="-DKEY_8B"; lib="-lsmj_hip_k8"; fi
    $CXX -x c++ -O2 -D_GNU_SOURCE -w $def $INC "$@" -x none -L"$LIB" $lib $RPATH \
        -lpthread -lm -o "$OUT/$name$w"
}
for w in 8 16; do
    build check_partitioning $w "$T/check_partitioning.c" "$T/testutil.c" $GEN
    build check_scalarsort $w "$T/check_scalarsort.c" "$T/testutil.c"
    build bench_partitioning $w "$S/bench/partitioningbench.c" $GEN "$S/util/memalloc.c"
    build bench_multiwaymerge $w "$S/bench/multiwaymergebench.c" "$T/testutil.c"
    build sortmergejoins $w "$S/main.c" $GEN "$S/util/memalloc.c" "$S/util/numa_shuffle.c"
    build tputbench $w "$S/bench/tputbench.c" $GEN "$S/util/memalloc.c" "$S/util/numa_shuffle.c"
    # main.c as built with --enable-materialize --enable-persist (Makefile.am:44-50):
    # R.tbl / S.tbl from the generators, the join output in Out.tbl
    build sortmergejoins_mat $w -DJOIN_MATERIALIZE -DPERSIST_RELATIONS "$S/main.c" $GEN \
        "$S/util/memalloc.c" "$S/util/numa_shuffle.c"
done
# sortbench.c sorts 8-byte items with avxsort_int64/avxsortmultiway_int64
buildxx bench_sort 8 "$S/bench/sortbench.c" "$T/testutil.c" $GEN
# avxsort only exists for 8-byte tuples (the reference forces scalar for 16 B)
build check_avxsort 8 "$T/check_avxsort.c" "$T/testutil.c"
# check_merge: 2-way, multiway (fan-in 2^2..2^11) and the AVX kernel tests,
# whose avxsort_core.h kernels map onto the device merge/sort
# (include/compat/avxsort_core.h)
build check_merge 8 "$T/check_merge.c" "$T/testutil.c"
echo "[build_dropin] built $(ls "$OUT" | wc -l) binaries in oracle/_ref/dropin"
