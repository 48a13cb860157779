#!/bin/bash
# The ~2 TB preset shard (240k x 256k + Laplacian, 20 iterations) at 64 and 128 frames on the final round-6 tree
export TMPDIR=/tmp
for nf in 64 128; do
  timeout -k 10 500 python -u bench.py --config 2tb --frames $nf --steps 2 --warmup 1 > gpurun_out/bench_r6_2tb_$nf.json 2> gpurun_out/bench_r6_2tb_$nf.err || { tail -20 gpurun_out/bench_r6_2tb_$nf.err; exit 1; }
  tail -1 gpurun_out/bench_r6_2tb_$nf.json | cut -c1-400
done
