export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_multiframe_bf16.py tests/test_gpu_multiframe.py tests/test_gpu_parity.py tests/test_gpu_realistic.py > gpurun_out/t21.log 2>&1 || { tail -30 gpurun_out/t21.log; exit 1; }
tail -2 gpurun_out/t21.log
for nf in 64 128; do
  timeout -k 10 240 python -u bench.py --steps 2 --warmup 1 --iters 100 --no-selfcheck --frames $nf > gpurun_out/mf_final_$nf.json 2> gpurun_out/mf_final_$nf.err || exit 1
done
timeout -k 10 240 python -u bench.py --steps 2 --warmup 1 --iters 100 --no-selfcheck --frames 64 --rtm-dtype bf16 > gpurun_out/mf_final_64b.json 2> gpurun_out/mf_final_64b.err || exit 1
timeout -k 10 400 python -u tools/parity_at_scale.py --no-bf16 --no-sparse --no-single --batches 64,128 --tag " r6 final2" --out gpurun_out/parity_r6_mf_final2.jsonl > gpurun_out/pmf2.log 2>&1
SART_LOAD_TRACE=1 timeout -k 10 300 python -u tools/sparse_load_rss.py --out gpurun_out/sparse_load_rss_r6e.jsonl > gpurun_out/srss5.log 2>&1
