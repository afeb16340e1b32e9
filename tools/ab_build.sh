#!/bin/bash
# A/B library: the in-tree objects with ONE source recompiled with extra flags.
#   tools/ab_build.sh <name> <source.hip> "<flags>"  ->  ab/libpaig_<name>.so
set -e
N=$1; SRC=$2; FL=$3
C=paig_reproduction_amd/csrc
mkdir -p ab/obj_$N
make -s -C $C >/dev/null
objs=$(ls $C/build/*.o | grep -v "/$(basename $SRC .hip).o$")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $FL -c $C/$SRC -o ab/obj_$N/x.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ab/libpaig_$N.so $objs ab/obj_$N/x.o
echo ab/libpaig_$N.so
