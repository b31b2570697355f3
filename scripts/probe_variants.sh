set -e
for sh in p1_8 p1_16 r256_8 r256_4 r128_32; do
  timeout -k 5 60 python scripts/conv_probe.py --shape $sh --iters 50
  DMC_NO_SPLITK=1 timeout -k 5 60 python scripts/conv_probe.py --shape $sh --iters 50 | sed 's/^/nosplit /'
  DMC_NO_BUFLDS=1 timeout -k 5 60 python scripts/conv_probe.py --shape $sh --iters 50 | sed 's/^/nobuf   /'
  DMC_NO_GLDS=1 timeout -k 5 60 python scripts/conv_probe.py --shape $sh --iters 50 | sed 's/^/noglds  /'
done
