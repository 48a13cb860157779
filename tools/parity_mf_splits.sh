#!/bin/bash
# The multi-frame engine's error at 64k x 64k against the fp32 two-pass kernels (tools/parity_at_scale.py) per operand
# split and per split-K count (accumulation-chain length): one run per environment below, 20 iterations, frame 0.
set -e
export TMPDIR=/tmp
out=${1:-gpurun_out/parity_r6_mf_splits.jsonl}
shift || true
variants=("$@")
[ ${#variants[@]} -eq 0 ] && variants=("" "SART_MF_BWD16=0" "SART_MF_FWD16=0" "SART_MF_X3=0")
for v in "${variants[@]}"; do
  env $v timeout -k 10 300 python -u tools/parity_at_scale.py --no-bf16 --no-sparse --no-single --batches 64 \
      --variants lin,log --frames 0 --iters 20 --tag " [$v]" --out "$out" >> "${out%.jsonl}.log" 2>&1
done
