#!/bin/bash
# Round 4, batch 8: the large-grid SW instances' shape (C4 all-sky: ring 9, a 2-wave floor with K = 3 or 4;
# C5 clear-sky: a 3-wave floor; the checkpoints of a column in one buffer range, C3 C4 C5), each SW solver alone against the default build, bitwise.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u tools/kernel_ab.py --config c4 --stage sw_solver --rounds 7 --iters 10 variants/big_r9.so variants/big_w2.so variants/big_k4w2.so variants/ckmerge.so > gpurun_out/r04/swbig_c4.txt 2>&1 || { tail -5 gpurun_out/r04/swbig_c4.txt; exit 1; }
grep sw_solver gpurun_out/r04/swbig_c4.txt
timeout -k 10 600 python -u tools/kernel_ab.py --config c5 --stage sw_solver --rounds 5 --iters 4 variants/nnw3.so variants/big_r9.so variants/big_r9_nnw3.so variants/ckmerge.so > gpurun_out/r04/swbig_c5.txt 2>&1 || { tail -5 gpurun_out/r04/swbig_c5.txt; exit 1; }
grep sw_solver gpurun_out/r04/swbig_c5.txt
timeout -k 10 300 python -u tools/kernel_ab.py --config c3 --stage sw_solver --rounds 9 --iters 20 variants/ckmerge.so > gpurun_out/r04/ckmerge_c3.txt 2>&1 || { tail -5 gpurun_out/r04/ckmerge_c3.txt; exit 1; }
grep sw_solver gpurun_out/r04/ckmerge_c3.txt
