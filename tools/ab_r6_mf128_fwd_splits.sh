export TMPDIR=/tmp
r() { tag=$1; shift; env "$@" timeout -k 10 240 python -u ab/fl0/bench.py --steps 2 --warmup 1 --iters 100 --no-selfcheck --frames 128 > gpurun_out/ab2_$tag.json 2>gpurun_out/ab2_$tag.err || exit 1; echo "$tag $(python3 -c "import json; d=json.loads(open('gpurun_out/ab2_$tag.json').read().strip().splitlines()[-1]); print(round(d['value']/17.179869184,1))")" | tee -a gpurun_out/ab2.txt; }
r fl0_def X=1
r fl0_fb4096 SART_MF_FWD_BLOCKS=4096
r fl0_fb8192 SART_MF_FWD_BLOCKS=8192
for fb in 4096 8192; do
SART_MF_FWD_BLOCKS=$fb timeout -k 10 300 python -u ab/fl0/tools/parity_at_scale.py --no-bf16 --no-sparse --no-single --batches 128 --variants lin,log --frames 0 --iters 20 --tag " fl0 fb$fb" --out gpurun_out/parity_ab2.jsonl >> gpurun_out/parity_ab2.log 2>&1 || exit 1
done
