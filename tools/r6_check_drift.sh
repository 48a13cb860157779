#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_multiframe.py -k drift > gpurun_out/t28.log 2>&1 || { tail -40 gpurun_out/t28.log; exit 1; }
tail -1 gpurun_out/t28.log
SART_LOAD_TRACE=1 timeout -k 10 300 python -u tools/sparse_load_rss.py --out gpurun_out/sparse_load_rss_r6f.jsonl > gpurun_out/srss6.log 2>&1
