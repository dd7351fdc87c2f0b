#!/bin/bash
# K sweep at fixed M x N: time(K) = per-tile fixed cost (prologue + epilogue) + K-proportional main loop.
for K in 256 512 768 1536 3072; do
  echo -n "K=$K nt256 "; python tools/gemm_one.py --op nt256 --M 50432 --N 3072 --K $K --iters 20 | tail -1
  echo -n "K=$K blas  "; python tools/gemm_one.py --op blas --M 50432 --N 3072 --K $K --iters 20 | tail -1
done
