# occupancy cost of an LDS landing zone in the fused layer backward (PAIG_BWD_LDS_PAD)
mkdir -p gpurun_out/r6u
for pad in 0 1024 24576 0 1024; do
  echo "pad=$pad" >> gpurun_out/r6u/bwd.txt
  PAIG_BWD_LDS_PAD=$pad timeout -k 10 120 python -u tools/bwd_bench.py c2,c10,c11,c12 1000 20 >> gpurun_out/r6u/bwd.txt 2>&1 || exit 1
done
