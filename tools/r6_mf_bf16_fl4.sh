#!/bin/bash
# bf16-storage forward without the second-level sums (tests + bench), and the split-A forward flushing every 4 trips
# (ab/freg4: bench at 64 / 128 frames and parity at 64k) against the product build
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_multiframe_bf16.py > gpurun_out/t23.log 2>&1 || { tail -30 gpurun_out/t23.log; exit 1; }
tail -1 gpurun_out/t23.log
b() { tag=$1; bench=$2; shift 2; timeout -k 10 240 python -u $bench --steps 2 --warmup 1 --iters 100 --no-selfcheck "$@" > gpurun_out/ab3_$tag.json 2> gpurun_out/ab3_$tag.err || exit 1; echo "$tag $(python3 -c "import json; d=json.loads(open('gpurun_out/ab3_$tag.json').read().strip().splitlines()[-1]); print(round(d['value']/17.179869184,1))")" | tee -a gpurun_out/ab3.txt; }
b base_64b bench.py --frames 64 --rtm-dtype bf16
b base_64 bench.py --frames 64
b base_128 bench.py --frames 128
b freg4_64 ab/freg4/bench.py --frames 64
b freg4_128 ab/freg4/bench.py --frames 128
b base_128b bench.py --frames 128 --rtm-dtype bf16
timeout -k 10 400 python -u ab/freg4/tools/parity_at_scale.py --no-bf16 --no-sparse --no-single --batches 64,128 --tag " freg4" --out gpurun_out/parity_freg4.jsonl > gpurun_out/pfreg4.log 2>&1
