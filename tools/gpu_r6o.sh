# decoder backward phase stamps (rollout + reconstruction, spring) and per-launch decoder times
mkdir -p gpurun_out/r6o
timeout -k 10 120 python -u tools/dec_bench.py 50 all > gpurun_out/r6o/dec_bench.txt 2>&1 || exit 1
PAIG_AB_LIB=paig_reproduction_amd/csrc/diag/libpaig_stamps.so timeout -k 10 120 python -u tools/dec_stamps.py spring_roll > gpurun_out/r6o/stamps_roll.txt 2>&1 || exit 1
PAIG_AB_LIB=paig_reproduction_amd/csrc/diag/libpaig_stamps.so timeout -k 10 120 python -u tools/dec_stamps.py spring_rec > gpurun_out/r6o/stamps_rec.txt 2>&1 || exit 1
