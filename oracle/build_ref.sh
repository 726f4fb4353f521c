#!/usr/bin/env bash
# Builds the CPU checker:
#   oracle/liboracle{8,16}.so      -- the in-repo C restatement (smj_oracle.c)
#   oracle/_ref/libref{8,16}.so    -- the REFERENCE itself, compiled from its
#                                     sources where they lie in /root/reference
#                                     plus oracle/ref_shim.cpp (C names)
#   oracle/_ref/cpu_baseline{8,16} -- reference m-way join timer (bench.py)
# Nothing is copied out of /root/reference; outputs go only to oracle/ and
# oracle/_ref/ (git-ignored, shipped to the GPU box with the tree).  When
# /root/reference is absent (the GPU box) only the restatement is built.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
REF="${SMJ_REFERENCE:-/root/reference}"
CC="${CC:-gcc}"
CXX="${CXX:-g++}"

for w in 8 16; do
    def=""; [ "$w" = 16 ] && def="-DKEY_8B"
    $CC -O2 -fPIC -shared $def "$HERE/smj_oracle.c" -o "$HERE/liboracle$w.so" -lm
done

if [ ! -d "$REF/src" ]; then
    echo "[build_ref] $REF not present: reference oracle not rebuilt"
    exit 0
fi
mkdir -p "$HERE/_ref"
S="$REF/src"
SRCS="$S/partition/partition.c $S/avxsort/avxsort.c $S/avxsort/avxsort_multiway.c \
 $S/merge/merge.c $S/merge/avx_multiwaymerge.c $S/merge/scalar_multiwaymerge.c \
 $S/scalarsort/scalarsort.c $S/joins/joincommon.c $S/joins/sortmergejoin_multiway.c \
 $S/datagen/generator.c $S/datagen/genzipf.c $S/util/cpu_mapping.c \
 $S/util/numa_shuffle.c $S/util/memalloc.c"
INC="-I$REF -I$S -I$S/partition -I$S/avxsort -I$S/merge -I$S/scalarsort -I$S/joins \
 -I$S/datagen -I$S/util"
# the fork needs C++ (src/avxsort/avxcommon.h:195-222 uses references)
FLAGS="-x c++ -O3 -mavx -DHAVE_AVX -D_GNU_SOURCE -DNDEBUG -fno-strict-aliasing -w -fPIC"
for w in 8 16; do
    def=""; [ "$w" = 16 ] && def="-DKEY_8B"
    objdir="$HERE/_ref/obj$w"; mkdir -p "$objdir"
    objs=""
    for f in $SRCS; do
        o="$objdir/$(basename "$f" .c).o"
        $CXX $FLAGS $def $INC -c "$f" -o "$o"
        objs="$objs $o"
    done
    $CXX -O2 -fPIC $def $INC -c "$HERE/ref_shim.cpp" -o "$objdir/ref_shim.o" -w
    # the AVX register kernels are inline in avxsort_core.h: a shim built -mavx
    $CXX $FLAGS $def $INC -c "$HERE/ref_shim_avx.cpp" -o "$objdir/ref_shim_avx.o"
    $CXX -shared -Wl,-Bsymbolic $objs "$objdir/ref_shim.o" "$objdir/ref_shim_avx.o" \
        -o "$HERE/_ref/libref$w.so" -lpthread -lm
    $CXX -O2 $def $INC -c "$HERE/cpu_baseline.cpp" -o "$objdir/cpu_baseline.o" -w
    $CXX $objs "$objdir/cpu_baseline.o" -o "$HERE/_ref/cpu_baseline$w" -lpthread -lm
    $CXX -O2 $def $INC -c "$HERE/cpu_baseline_ops.cpp" -o "$objdir/cpu_baseline_ops.o" -w
    $CXX $objs "$objdir/cpu_baseline_ops.o" -o "$HERE/_ref/cpu_baseline_ops$w" -lpthread -lm
    # the reference's own driver (src/main.c) on the reference objects: the
    # A side of tests/test_dropin.py's A/B run against oracle/_ref/dropin/
    for f in $S/joins/sortmergejoin_multipass.c $S/joins/sortmergejoin_mpsm.c $S/main.c; do
        $CXX $FLAGS $def $INC -c "$f" -o "$objdir/$(basename "$f" .c).o"
    done
    $CXX $objs "$objdir/sortmergejoin_multipass.o" "$objdir/sortmergejoin_mpsm.o" \
        "$objdir/main.o" -o "$HERE/_ref/sortmergejoins_ref$w" -lpthread -lm
    $CXX $FLAGS $def $INC -c "$S/bench/tputbench.c" -o "$objdir/tputbench.o"
    $CXX $objs "$objdir/tputbench.o" -o "$HERE/_ref/tputbench_ref$w" -lpthread -lm
done
echo "[build_ref] built oracle/_ref from $REF"
