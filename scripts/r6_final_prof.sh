#!/bin/bash
# round-6 profile set (same recipes as round 5): the bench line's roofline-conv kernel stats + FETCH/WRITE passes,
# DiT loop PMC, DDIM-50 / train kernel-trace summaries, the per-kernel roofline CSV of the eager train step and
# the graphed train step's kernel families
set -o pipefail
bash scripts/r5_benchprof.sh r6bp && bash scripts/r5_roofline.sh r6rf && bash scripts/r6_trace_train.sh r6tt
