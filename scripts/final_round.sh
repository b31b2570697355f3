#!/bin/bash
# end-of-session measurements: tests, bench, smoke, roofline stats + PMC, training / sampling / DiT traces,
# and the 2-rank gloo rehearsal of the multi-rank bench path. Each GPU step has its own limit; first failure ends.
set -e -o pipefail
export TMPDIR=/tmp
STAGES=tbsrmTSD bash scripts/gpu_round.sh r2f
bash scripts/rehearse_dp.sh r2f_rehearse
