#!/bin/bash
# Round-6 final-tree check: smoke(), the headline bench (driver contract, 20 steps), and a rocprofv3 kernel-stats pass
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6.log 2>&1 || { tail -20 gpurun_out/smoke_r6.log; exit 1; }
tail -3 gpurun_out/smoke_r6.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r6_headline.json 2> gpurun_out/bench_r6_headline.err || { tail -20 gpurun_out/bench_r6_headline.err; exit 1; }
tail -1 gpurun_out/bench_r6_headline.json
cd gpurun_out && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d prof_r6_head -o run -- python3 ../bench.py --steps 3 --warmup 1 > prof_r6_head.log 2>&1 || { tail -20 prof_r6_head.log; exit 1; }
find prof_r6_head -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} rocprof_r6_headline_kernel_stats.csv
find prof_r6_head -name "*.db" | head -1 | xargs -I{} python3 ../tools/trace_summary.py {} --marker k_fused_sweep_rows --top 8 > trace_r6_headline.txt 2>&1 || true
rm -rf prof_r6_head
