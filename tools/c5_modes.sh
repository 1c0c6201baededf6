# The C5 driver's three assignment modes through torch.distributed (NCCL, one rank on this box):
# frame-parallel LPT queue, tile-split + RCCL gather, static; an evenly spaced 10-frame sample.
# Output under gpurun_out/$TAG.
set -e
O=gpurun_out/${TAG:-c5_modes}; mkdir -p $O
F=${FRAMES:-0:300:30}
for m in frames tiles static; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29531 tools/animate.py --frames $F --split $m > $O/c5_$m.log 2>&1
  echo "$m done"
done
