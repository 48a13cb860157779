#!/bin/bash
# Runtime knobs of the split-A multi-frame kernels re-swept on the round-6 tree (two-level sums): frame-it/s, 64k x 64k
export TMPDIR=/tmp
for nf in ${NFS:-128 64}; do
  for kv in DEF=1 SART_MF_X3_DEPTH=3 SART_MF_H16=ew SART_MF_BP_BLOCKS=512 SART_MF_BP_BLOCKS=2048 SART_MF_FWD_BLOCKS=512 \
            SART_MF_FWD_BLOCKS=2048 SART_MF_X3_FWD=2,2,as SART_MF_X3_FWD=4,1,as DEF=1; do
    env $kv timeout -k 10 240 python -u bench.py --steps 2 --warmup 1 --iters 100 --no-selfcheck --frames $nf \
      > gpurun_out/knob.json 2> gpurun_out/knob.err || { tail -5 gpurun_out/knob.err; exit 1; }
    echo "$nf $kv $(python3 -c "import json; d=json.loads(open('gpurun_out/knob.json').read().strip().splitlines()[-1]); print(round(d['value']/17.179869184,1))")" | tee -a gpurun_out/knobs_r6.txt
  done
done
