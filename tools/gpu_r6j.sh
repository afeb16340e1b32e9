# fused layer backward phase stamps: real dY loads vs dY from a hot zero buffer (PAIG_BWD_NOLOAD)
mkdir -p gpurun_out/r6j
PAIG_AB_LIB=ab/libpaig_stamps.so timeout -k 10 120 python -u tools/bwd_bench.py c2,c7,c10,c11,c12 1000 20 > gpurun_out/r6j/stamps.txt 2>&1 || exit 1
PAIG_AB_LIB=ab/libpaig_stampsnl.so timeout -k 10 120 python -u tools/bwd_bench.py c2,c7,c10,c11,c12 1000 20 > gpurun_out/r6j/stamps_noload.txt 2>&1 || exit 1
