#!/bin/bash
# Build an experimental libbmh.so with extra compile flags for ONE source file, linked with the
# in-tree objects of the others: tools/build_variant.sh <name> <src.hip> <flags...>
# -> variants/<name>/libbmh.so (git-ignored; load it with BMH_LIB=variants/<name>/libbmh.so).
set -e
name=$1; src=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/bwt-mtf-huffman-compressor_amd
make -s -C "$pkg" >/dev/null
out=$root/variants/$name
mkdir -p "$out"
base=$(basename "$src")
# <src> is a csrc/ file name, or a path to another version of one (e.g. from git show)
[ -f "$src" ] && srcpath=$src || srcpath=$pkg/csrc/$base
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I"$root/include" --offload-arch=gfx950 \
    "$@" -I"$pkg/csrc" -c "$srcpath" -o "$out/$base.o"
objs=""
swapped=0
for o in "$pkg"/build/*.o; do
    if [ "$(basename "$o")" = "$base.o" ]; then
        objs="$objs $out/$base.o"
        swapped=1
    else
        objs="$objs $o"
    fi
done
# a source whose file name is no csrc/ file would leave the in-tree object in place
[ $swapped = 1 ] || { echo "build_variant: no csrc object $base.o (name the file like its csrc/ original)" >&2; exit 1; }
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$out/libbmh.so" $objs
echo "$out/libbmh.so"
