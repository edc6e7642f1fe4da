#!/bin/bash
# Build a variant of libasr_hip.so with one source recompiled under extra flags.
# usage: tools/build_variant.sh NAME SOURCE.hip "-DFLAG ..."   -> ablib/NAME/libasr_hip.so
set -e
NAME=$1; SRC=$2; FLAGS=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/pytorch_end2end_speech_recognition_amd/csrc
OUT=${VAR_DIR:-$ROOT/varlib}/$NAME   # varlib/ travels to the GPU box (git-ignored only)
mkdir -p $OUT/obj
BASE=$(basename $SRC .hip)
SLP=-fno-slp-vectorize   # as csrc/Makefile: SLP only in lstm_xg.hip
[ "$BASE" = lstm_xg ] && SLP=
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wall -Wno-unused-function -Wno-unused-variable $SLP $FLAGS -c $C/$SRC -o $OUT/obj/$BASE.o
OBJS=$(ls $C/build/*.o | grep -v "/$BASE.o$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libasr_hip.so $OBJS $OUT/obj/$BASE.o
rm -rf $OUT/obj
python3 $ROOT/tools/isa_check.py $OUT/libasr_hip.so
echo "built $OUT/libasr_hip.so"
