set -o pipefail
mkdir -p gpurun_out/r4t1
for shp in "128 32 128" "128 16 256" "128 8 256" "128 4 256"; do
  timeout -k 10 120 python -u scripts/dbg_gnbf.py $shp 2>&1 | grep -v amdgpu.ids || exit 1
done
