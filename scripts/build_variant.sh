#!/bin/bash
# Build varlibs/libhpe_<name>.so for GPU A/B runs (selected via HPE_LIB): the in-tree csrc/ with the
# given replacement sources, compiled by csrc/Makefile itself (same flags as the in-tree library).
# Usage: scripts/build_variant.sh <name> [<file.hip> ...] [-- <extra hipcc flags>]
# Each <file.hip> replaces the csrc/ file of the same basename (e.g. an older hpe_mlp2.hip saved
# as /tmp/x/hpe_mlp2.hip).  Objects whose sources are unchanged are reused from csrc/build.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/head-pose-estimation-model_amd/csrc
NAME=$1; shift
FILES=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do FILES+=("$1"); shift; done
[ "$1" = "--" ] && shift
make -C $CS -j8 >/dev/null
VD=$ROOT/head-pose-estimation-model_amd/var_$NAME   # sibling of csrc/: ../../include resolves
rm -rf $VD; mkdir -p $VD/build $ROOT/varlibs
cp -p $CS/*.hip $CS/*.h $CS/Makefile $VD/
cp -p $CS/build/*.o $VD/build/
touch $VD/build/*.o
for f in "${FILES[@]}"; do cp "$f" $VD/$(basename "$f"); touch $VD/$(basename "$f"); done
# extra flags: every object is rebuilt with them except the (slow) residual-stack kernels
[ $# -gt 0 ] && ls $VD/build/*.o | grep -v "hpe_res[0-9]" | xargs rm -f
make -C $VD -j8 OUT=$ROOT/varlibs/libhpe_$NAME.so EXTRA="$*" >/dev/null 2>$VD/build.err || { tail -20 $VD/build.err; exit 1; }
rm -rf $VD
echo built varlibs/libhpe_$NAME.so
