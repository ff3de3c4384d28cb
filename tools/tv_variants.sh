#!/bin/bash
# Build tuning variants of the codec library as
# stellatrain_amd/libstg_codec_<name>.so (only $SRC, default tv.hip, is recompiled):
#   [SRC=topk.hip] tools/tv_variants.sh name "-DSTG_TV_UNIT4=8192" [name2 "flags2" ...]
set -e
cd "$(dirname "$0")/../stellatrain_amd/csrc"
make -s -j8
while [ $# -ge 2 ]; do
    v=$1; f=$2; shift 2
    rm -rf build_$v && cp -a build build_$v && rm -f build_$v/${SRC:-tv.hip}.o
    make -s -j8 BUILD=build_$v OUT=../../tools/variants/libstg_codec_$v.so EXTRA="$f"
    echo "built libstg_codec_$v.so ($f)"
done
