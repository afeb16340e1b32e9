#!/bin/bash
# Diagnostic build of the decoder backward with s_memtime phase stamps
# (-DPAIG_DEC_STAMPS) linked with the other objects into build/libpaig_stamps.so.
set -e
cd "$(dirname "$0")/../paig_reproduction_amd/csrc"
make -s
mkdir -p build/stamps diag
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DPAIG_DEC_STAMPS -c decoder.hip -o build/stamps/decoder.o
objs=$(for f in *.hip; do b=${f%.hip}; [ "$b" != decoder ] && echo build/$b.o; done)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o diag/libpaig_stamps.so $objs build/stamps/decoder.o
echo built diag/libpaig_stamps.so
# phase-elimination variants (wrong results; timing only): pass 2 / pass 1 skipped
# (built only with DEC_SKIP=1)
[ "$DEC_SKIP" = 1 ] && for v in SKIP_P2 SKIP_P1; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DPAIG_DEC_$v -c decoder.hip -o build/stamps/decoder_$v.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o diag/libpaig_$v.so $objs build/stamps/decoder_$v.o
done
echo built diag variants
