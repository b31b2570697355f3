#!/bin/bash
# Halo conv variants and ablations on the UNet's halo shapes (conv_probe.py, HIP events on the launch stream).
# Ablation bits (DMC_HALO_DBG, LDS-DMA ring kernel only): 1 = no MFMA (VALU stand-in), 2 = no DMA in the loop,
# 4 = no LDS reads / MFMA (DMA + barriers only), 8 = no epilogue stores, 16 = s_setprio(1) around each MFMA
# cluster, 32 = static priority for waves 4-7, 64 = DMA issued after the first MFMA half of the stage.
# Variants: DMC_HALO_WS4=1 (4-slot weight ring), DMC_HALO_RW=1 (register-staged weights, one barrier per chunk).
# Stops at the first failure.
set -eo pipefail
P="timeout -k 10 60 python3 scripts/conv_probe.py --iters 50"
for b in 0 1 2 4 8 16 32 64; do
  echo "dbg=$b"
  DMC_HALO_DBG=$b $P --shape r128_32
done
for sh in r128_32 r384_32 r256_16 r512_8; do
  echo "ring3"; $P --shape $sh
  echo "ring4"; DMC_HALO_WS4=1 $P --shape $sh
  echo "regw"; DMC_HALO_RW=1 $P --shape $sh
done
