#!/bin/bash
# register epilogue everywhere (2) vs everywhere but the inference prologue halo kernel (3) vs off (0)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab11}
mkdir -p $O
REPS=2 bash scripts/ab.sh $O "DMC_REG_EPI=2" "DMC_REG_EPI=3" "DMC_REG_EPI=0"
