#!/bin/bash
# One parameterised A/B runner for a GPU box (replaces the per-experiment ab_*.sh scripts of round 2).
#
#   TESTS="-k halo_kernel" scripts/ab.sh OUTDIR "ENV1=a ENV2=b" "ENV1=c" ...
#
# 1. if TESTS is set: the GPU tests it selects (pytest args, e.g. "-k wgrad" or "tests/test_gpu_dit.py") run once
#    first (parity before timing);
# 2. one bench.py run per setting (BENCH_ARGS, default: the headline train + DDIM-50 + CFG lines), repeated
#    REPS times (default 1) in interleaved order so box drift hits every arm alike; one summary line per run.
# A setting may point DMC_LIB at another build of libdmc.so (e.g. the previous commit's) for a same-box regression.
set -e -o pipefail
export TMPDIR=/tmp
O=$1; shift
mkdir -p "$O"
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > "$O/tests.log" 2>&1 \
    || { tail -30 "$O/tests.log"; exit 1; }
  tail -1 "$O/tests.log"
fi
ARGS=${BENCH_ARGS:---no-extra --no-dit --no-cpu --no-roofline}
i=0
for rep in $(seq 1 ${REPS:-1}); do
  for cfg in "$@"; do
    i=$((i + 1))
    env $cfg timeout -k 10 300 python -u bench.py $ARGS > "$O/ab$i.json" 2> "$O/ab$i.err" || { tail -30 "$O/ab$i.err"; exit 1; }
    python3 - "$O/ab$i.json" "$cfg" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])   # RCCL prints a banner
parts = [f"train {d['value']}"] if d.get("value") else []
for k in ("ddim50", "ddim50_cfg"):
    if k in d:
        parts.append(f"{k} {d[k]['value']}")
if "dit_s2_ddim50_cfg" in d:
    parts.append(f"dit {d['dit_s2_ddim50_cfg']['value']} dit_train {d['dit_s2_ddim50_cfg'].get('train_img_s')}")
print(sys.argv[2].ljust(40), " ".join(parts))
PY
  done
done
