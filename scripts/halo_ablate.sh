#!/bin/bash
# Ablations of the halo conv kernel on the bench roofline shape: 1 = no MFMA (VALU stand-in), 2 = no DMA,
# 4 = no LDS reads / MFMA (DMA + barriers only), 8 = no epilogue stores.
for b in 0 1 2 4 8 6 9; do
  echo "dbg=$b"; DMC_HALO_DBG=$b timeout -k 10 60 python3 scripts/conv_probe.py --shape r128_32 --iters 50
done
