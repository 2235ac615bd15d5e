#!/bin/bash
# Sweep the split-K heuristic on the weight-gradient shapes (one process per setting).
for tgt in 256 512 1024; do
  for mk in 256 512 1024 2048; do
    echo "== target $tgt mink $mk"
    FDDM_SPLITK_TARGET=$tgt FDDM_SPLITK_MINK=$mk timeout -k 10 120 python tools/gemm_bench.py dw && timeout -k 10 120 python tools/gemm_bench.py dx || exit $?
  done
done
