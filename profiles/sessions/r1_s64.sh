# Collectives harness on the GPU path after the gloo-rehearsal change (world 1: RCCL launch and
# timing path only), then the bench under the DDP engine mode.
set -o pipefail
out=gpurun_out/s64
mkdir -p $out
timeout -k 10 180 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29564 tools/bench_collectives.py --json --min-mb 1 --max-mb 64 > $out/coll.log 2>&1 \
    || { tail -20 $out/coll.log; exit 1; }
grep '^{' $out/coll.log | tail -4
timeout -k 10 300 python -u bench.py --parallel ddp > $out/bench_ddp.log 2>&1 || { tail -20 $out/bench_ddp.log; exit 1; }
tail -1 $out/bench_ddp.log | cut -c1-260
