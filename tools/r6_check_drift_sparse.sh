#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_multiframe.py tests/test_gpu_sparse.py tests/test_native_driver.py > gpurun_out/t27.log 2>&1 || { tail -40 gpurun_out/t27.log; exit 1; }
tail -1 gpurun_out/t27.log
SART_LOAD_TRACE=1 timeout -k 10 300 python -u tools/sparse_load_rss.py --out gpurun_out/sparse_load_rss_r6f.jsonl > gpurun_out/srss6.log 2>&1
