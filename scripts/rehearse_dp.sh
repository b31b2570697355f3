# N=2 rehearsal of the multi-rank bench path on ONE GPU: two ranks share the card, gloo stages the all-reduces
# through the host (a plumbing check of GradSync + the segmented training graph, not a scaling number)
set -e -o pipefail
O=gpurun_out/${1:-rehearse}
mkdir -p "$O"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 4 --dist-backend gloo --no-cpu --no-cfg \
  > "$O/rehearse.json" 2> "$O/rehearse.err" || { tail -30 "$O/rehearse.err"; exit 1; }
cat "$O/rehearse.json"
