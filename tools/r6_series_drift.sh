#!/bin/bash
# Drift-extrapolated chain starts (SART_MF_DRIFT) on the 64k ray-traced series and its sparse version
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_multiframe.py > gpurun_out/t25.log 2>&1 || { tail -30 gpurun_out/t25.log; exit 1; }
tail -1 gpurun_out/t25.log
timeout -k 10 700 python -u tools/series_native.py --runs "${DENSE_RUNS:-batch64,batch64@SART_MF_DRIFT=1,batch64@SART_MF_DRIFT=0.5,batch64@SART_MF_DRIFT=1+SART_MF_SRC_AGE=5,batch64@SART_MF_DRIFT=1+SART_MF_SRC_AGE=8,batch128@SART_MF_DRIFT=1}" --out gpurun_out/series_drift.jsonl > gpurun_out/series_drift.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/series_native.py --sparse-direct --runs "${SPARSE_RUNS:-batch16,batch16@SART_MF_DRIFT=1,batch64@SART_MF_DRIFT=1}" --out gpurun_out/series_drift_sparse.jsonl > gpurun_out/series_drift_sparse.log 2>&1
