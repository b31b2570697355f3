#!/bin/bash
# dmc_gn_apply_fin: bitwise tests, then the same-box A/B (fused finalize-in-apply vs finalize + apply; DDIM with the
# halo prologue off, where every GroupNorm is materialised by the fused apply)
set -o pipefail
O=gpurun_out/${1:-r4af}
TESTS="-k fin tests/test_gpu_kernels.py tests/test_gpu_model.py" REPS=2 bash scripts/ab.sh $O \
  "DMC_GN_APPLY_FIN=1" "DMC_GN_APPLY_FIN=0" "DMC_GN_APPLY_FIN=1 DMC_HALO_PRO=0" "DMC_GN_APPLY_FIN=0 DMC_HALO_PRO=0"
