#!/bin/bash
# Same-box A/B of multi-frame builds (tools/ab_build.py variants under ab/<name>; "base" = the product build):
# bench.py frame-it/s at 64 / 128 frames (and bf16 storage at 64), 64k x 64k, 100 SART iterations per step.
# VARIANTS="base fregs flds4 base" bash tools/ab_r6_mf_flush.sh
export TMPDIR=/tmp
for v in ${VARIANTS:-base fregs flds4 base}; do
  b=bench.py; [ $v = base ] || b=ab/$v/bench.py
  for spec in ${SPECS:-64 128 64b}; do
    nf=${spec%b}; extra=""; [ $spec != $nf ] && extra="--rtm-dtype bf16"
    timeout -k 10 240 python -u $b --steps 2 --warmup 1 --iters 100 --no-selfcheck --frames $nf $extra \
      > gpurun_out/ab_${v}_$spec.json 2> gpurun_out/ab_${v}_$spec.err || exit 1
    echo "$v $spec $(python3 -c "import json; d=json.loads(open('gpurun_out/ab_${v}_$spec.json').read().strip().splitlines()[-1]); print(round(d['value']/17.179869184,1))")" | tee -a gpurun_out/ab_r6.txt
  done
done
