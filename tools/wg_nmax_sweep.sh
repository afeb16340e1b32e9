for n in 1024 512 256 128 64; do echo "NMAX $n"; PAIG_WG_NMAX=$n timeout -k 10 100 python tools/conv_bench.py 1000 split 20 c3,c4,c5,c6,c7,c8,c9,c2,c11 wgred || exit 1; done
