set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_r2
mkdir -p $O
timeout -k 10 60 python3 scripts/conv_probe.py --shape r128_32 --iters 20 > $O/probe.txt 2>&1
cat $O/probe.txt
bash scripts/pmc_conv.sh $O r128_32 > $O/pmc.log 2>&1
for d in sq sq2; do python3 scripts/pmc_summary.py $O/$d halo2; done
