# per-rank tile-split shares on one GPU (tools/rank_balance.py) + the RCCL bench path at N=1
set -e
O=gpurun_out/r02ae; mkdir -p $O
timeout -k 10 300 python tools/rank_balance.py c3 3 > $O/balance_c3.log 2>&1
timeout -k 10 300 python tools/rank_balance.py c2 3 > $O/balance_c2.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/torchrun_n1.json 2> $O/torchrun_n1.err
echo done
