#!/bin/bash
# Multi-frame throughput (bench.py, 100 SART iterations per step, 64k x 64k) per batch width and back-projection
# split target (SART_MF_BP_BLOCKS), and the engine's error at 64k for the same settings (tools/parity_at_scale.py)
set -e
export TMPDIR=/tmp
run() { tag=$1; shift; e=$1; shift; env $e timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --iters 100 --no-selfcheck "$@" \
    > gpurun_out/mfperf_$tag.json 2> gpurun_out/mfperf_$tag.err; }
for bp in ${BPS:-1024 2048 4096}; do
  run 64_bp$bp SART_MF_BP_BLOCKS=$bp --frames 64
  run 128_bp$bp SART_MF_BP_BLOCKS=$bp --frames 128
  SART_MF_BP_BLOCKS=$bp timeout -k 10 300 python -u tools/parity_at_scale.py --no-bf16 --no-sparse --no-single --batches 64 \
      --variants lin,log --frames 0 --iters 20 --tag " bp$bp" --out gpurun_out/parity_r6_mf_bp.jsonl >> gpurun_out/parity_r6_mf_bp.log 2>&1
done
