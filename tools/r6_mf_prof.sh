#!/bin/bash
# Kernel trace and one PMC pass of the 64- and 128-frame split-A sweeps on the final round-6 tree
export TMPDIR=/tmp
cd gpurun_out
for nf in 64 128; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d prof_mf$nf -o run -- python3 ../bench.py --steps 1 --warmup 0 --frames $nf --iters 20 --no-selfcheck > prof_mf$nf.log 2>&1 || { tail -20 prof_mf$nf.log; exit 1; }
  find prof_mf$nf -name "*.db" | head -1 | xargs -I{} python3 ../tools/trace_summary.py {} --marker k_mf_decide --top 10 > trace_r6_mf$nf.txt 2>&1 || true
  rm -rf prof_mf$nf
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d pmc_mf$nf -o run --output-format csv -- python3 ../bench.py --steps 1 --warmup 0 --frames $nf --iters 5 --no-selfcheck > pmc_mf$nf.log 2>&1 || { tail -20 pmc_mf$nf.log; exit 1; }
  find pmc_mf$nf -name "*counter_collection.csv" | head -1 | xargs -I{} cp {} pmc_r6_mf$nf.csv
  rm -rf pmc_mf$nf
done
