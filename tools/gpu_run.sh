#!/usr/bin/env bash
# GPU-box session script: each GPU step has its own time limit; a fault / abort / timeout ends the
# session (nothing else touches the GPU afterwards); ordinary test failures (exit 1) do not.
# Usage: tools/gpu_run.sh <step>...   steps: smoke tests testsall testsel(SEL=...) bench bench2 benchlog
#        probe probef prof
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0

run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))" | tee -a "$OUT/session.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -n 30 "$OUT/$name.log"
  case $rc in
    0|1|5) return 0 ;;          # success, test failures, no tests collected
    *) echo "FATAL step $name rc=$rc: stopping GPU session" | tee -a "$OUT/session.log"; exit $rc ;;
  esac
}

for step in "$@"; do
  case $step in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider ;;
    testsall) run pytest_gpu_all 1140 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    bench) run bench 600 python bench.py --steps 5 --warmup 1 ;;
    bench2) run bench_twopass 600 python bench.py --steps 5 --warmup 1 --no-fused ;;
    benchlog) run bench_log 600 python bench.py --steps 5 --warmup 1 --variant log ;;
    presets) run bench_512kx256k 600 python bench.py --config 512kx256k --steps 3 --warmup 1 &&
             run bench_2tb 900 python bench.py --config 2tb --steps 2 --warmup 1 &&
             run bench_256k 900 python bench.py --config 256k --steps 2 --warmup 1 ;;
    series) run series_fp32 600 python tools/series_bench.py --tol ${SERIES_TOL:-1e-8} &&
            run series_bf16 600 python tools/series_bench.py --dtype bf16 --batch 32 --tol ${SERIES_TOL:-1e-8} ;;
    probemfb) run probe_mfb16 900 python tools/probe_mf_b16.py ;;
    probemfx3) run probe_mfx3 900 python tools/probe_mf_x3.py ;;
    probeas) PROBE_DEPTH=2,3 PROBE_BWD=0 PROBE_FWD="2,2,lds;4,2,lds;2,2,lds,as;4,2,lds,as" \
               run probe_mfb_as 900 python tools/probe_mf_b16.py &&
             PROBE_FP32=0 PROBE_VT=1 PROBE_FWD="4,1;2,2;4,1,as;2,2,as;2,1,as;4,2,as" \
               run probe_mfx3_as 900 python tools/probe_mf_x3.py ;;
    benchmfx3) run bench_mfx32 600 python bench.py --steps 3 --warmup 1 --frames 32 &&
               run bench_mfx64 600 python bench.py --steps 3 --warmup 1 --frames 64 &&
               run bench_mff64 600 python bench.py --steps 3 --warmup 1 --frames 64 --mf-split-a off ;;
    probemfbv) PROBE_DEPTH=2,3 PROBE_FWD="2,2,lds;4,2,lds" run probe_mfb_bwd 900 python tools/probe_mf_b16.py ;;
    probemfbl) PROBE_BWD=0 PROBE_DEPTH=2,3 PROBE_FWD="4,2;8,1;4,1,lds;4,2,lds;8,1,lds;2,2,lds" \
                 run probe_mfb_lds 900 python tools/probe_mf_b16.py ;;
    benchmfb) run bench_mfb16 600 python bench.py --steps 3 --warmup 1 --frames 16 --rtm-dtype bf16 &&
              run bench_mfb32 600 python bench.py --steps 3 --warmup 1 --frames 32 --rtm-dtype bf16 &&
              run bench_mfb64 600 python bench.py --steps 3 --warmup 1 --frames 64 --rtm-dtype bf16 ;;
    benchmf) run bench_mf16 600 python bench.py --steps 3 --warmup 1 --frames 16 &&
             run bench_mf32 600 python bench.py --steps 3 --warmup 1 --frames 32 &&
             run bench_mf64 600 python bench.py --steps 3 --warmup 1 --frames 64 ;;
    mfdepth) for d in 1 2 3; do for nf in 16 32 64; do
               SART_MF_DEPTH=$d run bench_mf${nf}_d$d 300 python bench.py --steps 2 --warmup 1 --frames $nf --iters 50 || exit 1
             done; done ;;
    profx3) run rocprof_x3_64 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_x3_64" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames 64 --iters 20 &&
            run rocprof_x3_32 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_x3_32" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames 32 --iters 20 ;;
    cfg1) run config1_blocked 300 python tools/cpu_config1.py --ranks 1,4 --out "$OUT/config1.jsonl" &&
          SART_CPU_TWO_PASS=1 run config1_twopass 300 python tools/cpu_config1.py --ranks 1,4 --out "$OUT/config1_twopass.jsonl" &&
          run config1_blocked2 300 python tools/cpu_config1.py --ranks 1,4 --gpu --out "$OUT/config1.jsonl" ;;
    profhead) run rocprof_head 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_head" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 ;;
    profmf128) for nf in 64 128; do
              run rocprof_mfx$nf 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_mfx$nf" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames $nf --iters 20 --no-selfcheck || exit 1
            done ;;
    r5mf) for cfg in "64|fp32" "128|fp32" "64|bf16" "128|bf16" "32|fp32"; do
            nf=${cfg%%|*}; dt=${cfg#*|}
            run bench_r5_mf${nf}_$dt 300 python bench.py --steps 3 --warmup 1 --frames $nf --rtm-dtype $dt || exit 1
            grep -h '^{' "$OUT/bench_r5_mf${nf}_$dt.log" >> "$OUT/bench_r5_mf.jsonl"
          done ;;
    r52tb) for nf in 64 128; do
             run bench_r5_2tb_$nf 900 python bench.py --config 2tb --steps 2 --warmup 1 --frames $nf || exit 1
             grep -h '^{' "$OUT/bench_r5_2tb_$nf.log" >> "$OUT/bench_r5_mf.jsonl"
           done ;;
    splitchk) run split_h2_check 120 tools/split_h2_check &&
              run pytest_mf16 900 python -u -m pytest tests/test_gpu_realistic.py tests/test_gpu_multiframe_bf16.py -m gpu -x -q \
                -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    abmix)  # split_h2 on v_fma_mix (new) vs the C++ split (.abold), same box, alternating
      for i in 1 2; do
        for cfg in ${AB_CFGS:-64| 128| 64|--config=2tb}; do  # one token per config: frames|extra-argument
          nf=${cfg%%|*}; ex=${cfg#*|}; tag=${nf}${ex:+_${ex##*=}}
          timeout -k 10 600 python .abold/bench.py --steps 3 --warmup 1 --frames $nf $ex --no-selfcheck > "$OUT/abmix_old_${tag}_$i.log" 2>&1 &&
          timeout -k 10 600 python bench.py --steps 3 --warmup 1 --frames $nf $ex --no-selfcheck > "$OUT/abmix_new_${tag}_$i.log" 2>&1 || { echo "FATAL $tag"; exit 1; }
          echo "=== abmix $tag $i old $(grep -h '^{' "$OUT/abmix_old_${tag}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"])') new $(grep -h '^{' "$OUT/abmix_new_${tag}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"])')" | tee -a "$OUT/session.log"
        done
      done ;;
    abdepth)  # register-ring depth of the f16-pair kernels: forward (SART_MF_H16_FDEPTH) / back-projection (SART_MF_X3_DEPTH)
      for i in 1 2; do
        for nf in 64 128; do
          for cfg in "2,2" "3,2" "2,3" "3,3"; do
            fd=${cfg%%,*}; bd=${cfg#*,}
            SART_MF_H16_FDEPTH=$fd SART_MF_X3_DEPTH=$bd timeout -k 10 300 python bench.py --steps 3 --warmup 1 --frames $nf --no-selfcheck \
              > "$OUT/abd_${nf}_${fd}${bd}_$i.log" 2>&1 || { echo "FATAL $nf $cfg"; exit 1; }
            echo "=== abdepth nf=$nf fwd=$fd bwd=$bd $i $(grep -h '^{' "$OUT/abd_${nf}_${fd}${bd}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"])')" | tee -a "$OUT/session.log"
          done
        done
      done ;;
    abenv)  # env-knob A/B on one build: AB_RUNS = "tag|frames|extra-arg|ENV=VAL[;ENV=VAL]" tokens, two rounds
      for i in 1 2; do
        for r in $AB_RUNS; do
          IFS='|' read -r tag nf ex ev <<< "$r"
          env ${ev//;/ } timeout -k 10 300 python bench.py --steps 3 --warmup 1 --frames $nf $ex --no-selfcheck > "$OUT/abenv_${tag}_$i.log" 2>&1 || { echo "FATAL $tag"; exit 1; }
          echo "=== abenv $tag $i $(grep -h '^{' "$OUT/abenv_${tag}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])')" | tee -a "$OUT/session.log"
        done
      done ;;
    prof64) run rocprof_mfx64b 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_mfx64b" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames 64 --iters 20 --no-selfcheck &&
            run rocprof_2tb64 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_2tb64" -o run --output-format csv -- python3 bench.py --config 2tb --steps 1 --warmup 0 --frames 64 --no-selfcheck ;;
    sparse) run pytest_sparse 900 python -u -m pytest tests/test_gpu_sparse.py tests/test_cli_e2e.py tests/test_native_driver.py \
              -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    sparsebench) run sparse_bench 600 python tools/sparse_bench.py --frames 16,32,64,128 --out "$OUT/sparse_bench.jsonl" ;;
    sparsepw)  # SpMM plane width (SART_MF_SPARSE_PW) by batch width, two rounds
      for i in 1 2; do for pw in 64 32 16; do
        SART_MF_SPARSE_PW=$pw run sparse_pw_${pw}_$i 300 python tools/sparse_bench.py --no-dense --frames 32,64,128 \
          --out "$OUT/sparse_pw_${pw}_$i.jsonl"
      done; done ;;
    profsparsemf) for nf in 16 64; do
        run rocprof_sparse_mf$nf 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_sparse_mf$nf" -o run --output-format csv \
          -- python3 tools/sparse_bench.py --no-dense --steps 2 --frames $nf || exit 1
      done ;;
    sparselanes) for l in 4 8 16 32; do
                   SART_SPARSE_LANES=$l run sparse_lanes_$l 300 python tools/sparse_bench.py --no-dense --out "$OUT/sparse_lanes_$l.jsonl" || exit 1
                 done
                 run sparse_lanes_auto 300 python tools/sparse_bench.py --no-dense --out "$OUT/sparse_lanes_auto.jsonl" &&
                 run rocprof_sparse 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_sparse" -o run --output-format csv -- python3 tools/sparse_bench.py --no-dense --steps 2 ;;
    seriessparse) run series_sparse 900 python tools/series_native.py --sparse-direct --runs ${SERIES_RUNS:-seq} --out "$OUT/series_sparse.jsonl" ;;
    seriesdense) run series_dense 900 python tools/series_native.py --runs ${SERIES_RUNS:-seq} --out "$OUT/series_dense.jsonl" ;;
    sparsedens) for d in 0.01 0.03 0.05 0.1 0.2; do
                  run sparse_dens_$d 600 python tools/sparse_bench.py --random-density $d --shape 128,128 --grid 32,32,32 \
                    --out "$OUT/sparse_density.jsonl" || exit 1
                done ;;
    profmfb) for nf in 16 64; do
              run rocprof_mfb$nf 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_mfb$nf" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames $nf --iters 20 --rtm-dtype bf16 || exit 1
            done ;;
    profmf) for nf in 16 32 64; do
              run rocprof_mf$nf 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_mf$nf" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames $nf --iters 20 || exit 1
            done ;;
    mfoverlap)  # 2 ranks on one GPU, each under its own rocprofv3 (no launcher between profiler and python)
      port=$(python -c 'import socket; s = socket.socket(); s.bind(("127.0.0.1", 0)); print(s.getsockname()[1])')
      echo "=== mfoverlap ($(date +%T))" | tee -a "$OUT/session.log"
      pids=()
      for r in 0 1; do
        MASTER_ADDR=127.0.0.1 MASTER_PORT=$port RANK=$r WORLD_SIZE=2 LOCAL_RANK=$r LOCAL_WORLD_SIZE=2 \
          SART_DIST_BACKEND=gloo SART_P2P=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/mfov_r$r" -o run \
          --output-format csv -- python3 tools/dist_check.py --multiframe --batch 32 --npix 8192 --nvox 65536 \
          --iters 20 --out "$OUT/mfov" > "$OUT/mfov_r$r.log" 2>&1 &
        pids+=($!)
      done
      rc=0
      for p in "${pids[@]}"; do wait "$p" || rc=$?; done
      echo "=== mfoverlap rc=$rc" | tee -a "$OUT/session.log"
      [ $rc -eq 0 ] || { tail -n 20 "$OUT"/mfov_r*.log; exit $rc; }
      for r in 0 1; do
        python tools/overlap_report.py "$(ls "$OUT"/mfov_r$r/*/run_kernel_trace.csv "$OUT"/mfov_r$r/run_kernel_trace.csv 2>/dev/null | head -n 1)" \
          --out "$OUT/mfov_report_r$r.json" || true
      done ;;
    benchshare) run bench_share2 600 python bench.py --gpus 2 --share-gpus --steps 3 --warmup 1 ;;
    cw8) run fcheck_cw8 600 python tools/fused_check.py 8192x300000 4096x150528 &&
         for i in 1 2; do
           for v in 300000 530432; do
             SART_FUSED_CW_SCHED=5 run bench_cw5_${v}_$i 300 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck &&
             run bench_cw8_${v}_$i 300 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck || exit 1
           done
         done ;;
    kw5) SART_FUSED_KW5=1 run fcheck_kw5 600 python tools/fused_check.py 4096x150000 4096x163840 &&
         SART_FUSED_KW5=1 SART_FUSED_XL_SCHED=8 run fcheck_kw5s8 600 python tools/fused_check.py 4096x150000 4096x200000 &&
         for i in 1 2; do
           for v in 147456 150000 155648 163840; do
             run bench_kwb_${v}_$i 300 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck &&
             SART_FUSED_KW5=1 run bench_kw5_${v}_$i 300 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck &&
             SART_FUSED_KW5=1 SART_FUSED_XL_SCHED=8 run bench_kw5s8_${v}_$i 300 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck || exit 1
           done
           for v in 100000 200000; do
             run bench_kwb_${v}_$i 300 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck &&
             SART_FUSED_XL_SCHED=8 run bench_kws8_${v}_$i 300 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck || exit 1
           done
         done ;;
    rsab) SART_FUSED_KW5=1 run fcheck_rs 600 python tools/fused_check.py 4096x150000 4096x200000 4096x100000 4096x300000 &&
          for i in 1 2; do
            for cfg in 150000: 150000:SART_FUSED_KW5=1 163840:SART_FUSED_KW5=1 200000: 100000: 300000: 524288: 65536:; do
              v=${cfg%%:*}; e=${cfg#*:}; tag=${v}_${e:+kw5}
              env $e timeout -k 10 300 python .abold/bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/rs_old_${tag}_$i.log" 2>&1 &&
              env $e timeout -k 10 300 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/rs_new_${tag}_$i.log" 2>&1 || exit 1
              echo "=== rs $tag $i old $(grep -o '"effective_hbm_TBps_per_gpu": [0-9.]*' "$OUT/rs_old_${tag}_$i.log") new $(grep -o '"effective_hbm_TBps_per_gpu": [0-9.]*' "$OUT/rs_new_${tag}_$i.log")" | tee -a "$OUT/session.log"
            done
          done ;;
    mfminw) for i in 1 2; do
              timeout -k 10 300 python .abold/bench.py --steps 3 --warmup 1 --no-selfcheck --frames 64 --rtm-dtype bf16 > "$OUT/mfw_old_$i.log" 2>&1 || exit 1
              echo "=== mfw old $i $(grep -h '^{' "$OUT/mfw_old_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])')" | tee -a "$OUT/session.log"
              for cfg in "2|4,2,lds|1,lds" "3|4,1,lds|1,lds" "3|2,2,lds|1,lds" "2|2,2,lds|1,lds" "2|4,2,lds|2,lds"; do
                d=${cfg%%|*}; rest=${cfg#*|}; f=${rest%%|*}; v=${rest#*|}
                SART_MF_DEPTH=$d SART_MF_B16_FWD=$f SART_MF_B16_VT=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-selfcheck --frames 64 --rtm-dtype bf16 > "$OUT/mfw_new_${d}_${f}_${v}_$i.log" 2>&1 || exit 1
                echo "=== mfw new d=$d fwd=$f vt=$v $i $(grep -h '^{' "$OUT/mfw_new_${d}_${f}_${v}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])')" | tee -a "$OUT/session.log"
              done
            done ;;
    small3) for p in 8192 16384; do
              run bench_small_$p 300 python bench.py --steps 5 --warmup 1 --npix $p --no-selfcheck || exit 1
            done ;;
    rehearse8f) SART_P2P_TIMEOUT_S=60 run bench_share8_fused 500 python bench.py --gpus 8 --share-gpus --npix 16384 \
                  --steps 3 --warmup 1 --watchdog 300 ;;
    widths3) for v in 150000 200000 100000 300000 524288; do
               run bench_w3_$v 300 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck &&
               SART_FUSED_XL=1 run bench_w3xl_$v 300 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck || exit 1
             done &&
             run bench_w3_1m 300 python bench.py --steps 3 --warmup 1 --nvox 1048576 --npix 16384 --no-selfcheck &&
             SART_FUSED_XL=1 run bench_w3xl_1m 300 python bench.py --steps 3 --warmup 1 --nvox 1048576 --npix 16384 --no-selfcheck ;;
    widthsweep)  # 65536 rows x 32768 ... 262144 voxels in steps of 8192 (one JSON line per width)
      for v in $(seq ${WS_FROM:-32768} 8192 ${WS_TO:-262144}); do
        timeout -k 10 200 python bench.py --steps 3 --warmup 1 --iters ${WS_ITERS:-50} --nvox $v --no-selfcheck \
          > "$OUT/ws_$v.log" 2>&1 || { echo "FATAL width $v"; tail -n 20 "$OUT/ws_$v.log"; exit 1; }
        grep -h '^{' "$OUT/ws_$v.log" >> "$OUT/widthsweep.jsonl"
        echo "=== width $v $(grep -h '^{' "$OUT/ws_$v.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], d["fused_grid"])')" | tee -a "$OUT/session.log"
      done ;;
    mfdeep)  # bf16 64-frame ring depth A/B (3 = default, 4, 5) + the MF bf16 tests at depth 5
      SART_MF_DEPTH=5 run pytest_mfdeep 600 python -u -m pytest tests/test_gpu_multiframe_bf16.py -m gpu -x -q \
        -p no:cacheprovider --timeout 120 --timeout-method thread &&
      for i in 1 2; do
        for d in 3 4 5; do
          SART_MF_DEPTH=$d timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-selfcheck --frames 64 --rtm-dtype bf16 \
            > "$OUT/mfd_${d}_$i.log" 2>&1 || { echo "FATAL depth $d"; tail -n 20 "$OUT/mfd_${d}_$i.log"; exit 1; }
          echo "=== mfdeep d=$d run $i $(grep -h '^{' "$OUT/mfd_${d}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])')" | tee -a "$OUT/session.log"
        done
      done ;;
    pmcfetchmf)  # HBM bytes per multi-frame kernel (bf16 shard, 64 frames): is X / W re-read from memory?
      echo "=== pmcfetchmf" >> "$OUT/session.log"
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_mfb64" -o run --output-format csv -- python3 bench.py \
        --steps 1 --warmup 0 --frames 64 --iters 5 --rtm-dtype bf16 --no-selfcheck > "$OUT/pmc_fetch_mfb64.log" 2>&1
      rc=$?; echo "=== pmcfetchmf rc=$rc" >> "$OUT/session.log"; [ $rc -eq 0 ] || exit $rc ;;
    probes3) run probe_mf_ld 300 python tools/probe_mf_ld.py &&
             run ablation_dips 300 python tools/fused_ablation.py --dtype fp32 65536x147456 65536x172032 65536x73728 65536x139264 ;;
    abt1)  # T = 1 register-ring depth by slab width (new) vs 4 tiles at every kw (.abold), kw 5 opt-in
      run pytest_t1 600 python -u -m pytest tests/test_gpu_solver.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
      SART_FUSED_KW5=1 run fcheck_t1kw5 300 python tools/fused_check.py 4096x150000 4096x163840 8192x147456 &&
      for i in 1 2; do
        for cfg in 147456: 163840: 180224: 100000: 200000: 300000: 65536: 150000:SART_FUSED_KW5=1 163840:SART_FUSED_KW5=1; do
          v=${cfg%%:*}; e=${cfg#*:}; tag=${v}${e:+_kw5}
          env $e timeout -k 10 200 python .abold/bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/t1_old_${tag}_$i.log" 2>&1 &&
          env $e timeout -k 10 200 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/t1_new_${tag}_$i.log" 2>&1 || { echo "FATAL $tag"; exit 1; }
          echo "=== t1 $tag $i old $(grep -h '^{' "$OUT/t1_old_${tag}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], d["fused_grid"])') new $(grep -h '^{' "$OUT/t1_new_${tag}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])')" | tee -a "$OUT/session.log"
        done
      done ;;
    access) run access_probe 120 tools/access_probe 0 && run access_probe_pitch 120 tools/access_probe 256 ;;
    abkw9)  # 9-KiB T = 1 slabs (new default where cheaper) vs SART_FUSED_KW9=0; ring depth vs .abold (4 tiles at every kw)
      run fcheck_kw9 300 python tools/fused_check.py 4096x147456 4096x73728 4096x294912 8192x70000 &&
      SART_FUSED_KW5=1 run fcheck_kw5b 300 python tools/fused_check.py 4096x150000 &&
      SEL="tests/test_gpu_solver.py" run pytest_kw9 600 python -u -m pytest tests/test_gpu_solver.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
      for i in 1 2; do
        for v in 70000 73728 90112 139264 147456 294912; do
          timeout -k 10 200 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/k9_new_${v}_$i.log" 2>&1 &&
          SART_FUSED_KW9=0 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/k9_off_${v}_$i.log" 2>&1 || { echo "FATAL $v"; exit 1; }
          echo "=== kw9 $v $i on $(grep -h '^{' "$OUT/k9_new_${v}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], d["fused_grid"])') off $(grep -h '^{' "$OUT/k9_off_${v}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], d["fused_grid"])')" | tee -a "$OUT/session.log"
        done
        for cfg in 147456:SART_FUSED_KW9=0 163840: 200000: 65536: 150000:SART_FUSED_KW5=1; do
          v=${cfg%%:*}; e=${cfg#*:}; tag=${v}${e:+_${e#SART_FUSED_}}
          if [ "$e" != "SART_FUSED_KW5=1" ]; then
            env $e timeout -k 10 200 python .abold/bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/rd_old_${tag}_$i.log" 2>&1 || { echo "FATAL old $tag"; exit 1; }
          fi
          env $e timeout -k 10 200 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/rd_new_${tag}_$i.log" 2>&1 || { echo "FATAL new $tag"; exit 1; }
          echo "=== ring $tag $i old $(grep -sh '^{' "$OUT/rd_old_${tag}_$i.log" | python -c 'import sys,json; l=sys.stdin.readline(); d=json.loads(l) if l else {}; print(d.get("iters_per_s"), d.get("effective_hbm_TBps_per_gpu"))') new $(grep -h '^{' "$OUT/rd_new_${tag}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], d["fused_grid"])')" | tee -a "$OUT/session.log"
        done
      done ;;
    ablpub)  # T = 1 lane-partial publication (new) vs the wave_sum in every compute wave (.abold)
      run fcheck_lpub 300 python tools/fused_check.py 4096x131072 4096x150000 4096x147456 4096x300000 8192x262144 &&
      SART_FUSED_KW5=1 run fcheck_lpub5 300 python tools/fused_check.py 4096x163840 &&
      run pytest_lpub 600 python -u -m pytest tests/test_gpu_solver.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
      for i in 1 2; do
        for cfg in 155648: 163840: 180224: 150000: 147456: 262144: 300000: 100000: 150000:SART_FUSED_KW5=1 163840:SART_FUSED_KW5=1; do
          v=${cfg%%:*}; e=${cfg#*:}; tag=${v}${e:+_kw5}
          env $e timeout -k 10 200 python .abold/bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/lp_old_${tag}_$i.log" 2>&1 &&
          env $e timeout -k 10 200 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/lp_new_${tag}_$i.log" 2>&1 || { echo "FATAL $tag"; exit 1; }
          echo "=== lpub $tag $i old $(grep -h '^{' "$OUT/lp_old_${tag}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])') new $(grep -h '^{' "$OUT/lp_new_${tag}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], d["fused_grid"])')" | tee -a "$OUT/session.log"
        done
      done ;;
    abflag4)  # one 16-byte LDS read for a slot's four wave flags / partials (new) vs four polls in turn (.abold)
      run fcheck_flag4 300 python tools/fused_check.py 4096x131072 4096x150000 4096x147456 4096x300000 16384x65536 &&
      run fcheck_flag4_old 300 python .abold/tools/fused_check.py 4096x131072 4096x150000 4096x147456 4096x300000 16384x65536 &&
      run pytest_flag4 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_bf16.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
      for i in 1 2; do
        for v in 150000 163840 188416 100000 200000 262144 300000 524288 65536 98304; do
          timeout -k 10 200 python .abold/bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/f4_old_${v}_$i.log" 2>&1 &&
          timeout -k 10 200 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/f4_new_${v}_$i.log" 2>&1 || { echo "FATAL $v"; exit 1; }
          echo "=== flag4 $v $i old $(grep -h '^{' "$OUT/f4_old_${v}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])') new $(grep -h '^{' "$OUT/f4_new_${v}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], d["fused_grid"])')" | tee -a "$OUT/session.log"
        done
      done ;;
    kw5b)  # 5-KiB slabs (with the 16-byte flag reads) against the default geometry at the kw 6 widths with idle CUs
      for i in 1 2; do
        for v in 150000 155648 163840 147456; do
          timeout -k 10 200 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/k5_def_${v}_$i.log" 2>&1 &&
          SART_FUSED_KW5=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/k5_on_${v}_$i.log" 2>&1 || { echo "FATAL $v"; exit 1; }
          echo "=== kw5b $v $i def $(grep -h '^{' "$OUT/k5_def_${v}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], d["fused_grid"])') kw5 $(grep -h '^{' "$OUT/k5_on_${v}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], d["fused_grid"])')" | tee -a "$OUT/session.log"
        done
      done ;;
    abstage)  # multi-frame bf16 / split-A kernels: next step's X / W staged after the MFMAs (new) vs before (.abold)
      run pytest_stage 600 python -u -m pytest tests/test_gpu_multiframe.py tests/test_gpu_multiframe_bf16.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
      for i in 1 2; do
        for spec in "b64|--frames 64 --rtm-dtype bf16" "f64|--frames 64" "b32|--frames 32 --rtm-dtype bf16" "f32|--frames 32" "b16|--frames 16 --rtm-dtype bf16"; do
          name=${spec%%|*}; args=${spec#*|}
          timeout -k 10 300 python .abold/bench.py --steps 3 --warmup 1 --no-selfcheck $args > "$OUT/st_old_${name}_$i.log" 2>&1 &&
          timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-selfcheck $args > "$OUT/st_new_${name}_$i.log" 2>&1 || { echo "FATAL $name"; exit 1; }
          echo "=== stage $name $i old $(grep -h '^{' "$OUT/st_old_${name}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])') new $(grep -h '^{' "$OUT/st_new_${name}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])')" | tee -a "$OUT/session.log"
        done
      done ;;
    prof2tb) run rocprof_2tb 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_2tb" -o run --output-format csv -- python3 bench.py --config 2tb --steps 1 --warmup 0 --no-selfcheck &&
             run rocprof_mfx64 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_mfx64" -o run --output-format csv -- python3 bench.py --frames 64 --steps 1 --warmup 0 --iters 20 --no-selfcheck ;;
    finalb) run bench_bf16 300 python bench.py --steps 5 --warmup 1 --rtm-dtype bf16 &&
            run bench_mfb64 300 python bench.py --steps 3 --warmup 1 --frames 64 --rtm-dtype bf16 &&
            run bench_mfx64 300 python bench.py --steps 3 --warmup 1 --frames 64 &&
            run bench_mfx32 300 python bench.py --steps 3 --warmup 1 --frames 32 &&
            run bench_2tb 600 python bench.py --config 2tb --steps 2 --warmup 1 &&
            run bench_512k 600 python bench.py --config 512kx256k --steps 3 --warmup 1 ;;
    cw9) SART_FUSED_XL=0 run fcheck_cw9 300 python tools/fused_check.py 4096x368640 &&
         for i in 1 2; do
           for v in 368640 385024; do
             timeout -k 10 200 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/cw9_on_${v}_$i.log" 2>&1 &&
             SART_FUSED_KW9=0 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/cw9_off_${v}_$i.log" 2>&1 || { echo "FATAL $v"; exit 1; }
             echo "=== cw9 $v $i on $(grep -h '^{' "$OUT/cw9_on_${v}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], d["fused_grid"])') off $(grep -h '^{' "$OUT/cw9_off_${v}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], d["fused_grid"])')" | tee -a "$OUT/session.log"
           done
         done ;;
    abkw8)  # 8-KiB T = 1 slabs across builds: HEAD / pre-flag4 (.abold) / round-3 start (.abr3s), same box, interleaved
      for i in 1 2; do
        for v in 262144 131072; do
          for b in head old r3s; do
            case $b in head) py=bench.py ;; old) py=.abold/bench.py ;; r3s) py=.abr3s/bench.py ;; esac
            timeout -k 10 200 python $py --steps 3 --warmup 1 --nvox $v --no-selfcheck > "$OUT/k8_${b}_${v}_$i.log" 2>&1 || { echo "FATAL $b $v"; exit 1; }
          done
          echo "=== kw8 $v $i $(for b in head old r3s; do echo -n "$b "; grep -h '^{' "$OUT/k8_${b}_${v}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], end=" ")'; done)" | tee -a "$OUT/session.log"
        done
      done ;;
    mfnw)  # 64-frame bf16 kernels: 8 waves of half-size tiles (SART_MF_B16_NW=8) vs 4 waves
      SART_MF_B16_NW=8 run pytest_mfnw 600 python -u -m pytest tests/test_gpu_multiframe_bf16.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
      for i in 1 2; do
        timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-selfcheck --frames 64 --rtm-dtype bf16 > "$OUT/nw4_$i.log" 2>&1 &&
        SART_MF_B16_NW=8 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-selfcheck --frames 64 --rtm-dtype bf16 > "$OUT/nw8_$i.log" 2>&1 || { echo "FATAL nw"; exit 1; }
        echo "=== mfnw $i nw4 $(grep -h '^{' "$OUT/nw4_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])') nw8 $(grep -h '^{' "$OUT/nw8_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])')" | tee -a "$OUT/session.log"
      done ;;
    fwd2tb)  # forward split-K count at the 2tb preset shard (245760 x 262144, 64 frames split-A)
      for kv in DEF=0 SART_MF_FWD_BLOCKS=2048 SART_MF_FWD_BLOCKS=4096 SART_MF_FWD_BLOCKS=8192; do
        env "$kv" timeout -k 10 400 python bench.py --config 2tb --steps 1 --warmup 1 --no-selfcheck > "$OUT/f2tb_$kv.log" 2>&1 || { echo "FATAL $kv"; exit 1; }
        echo "=== fwd2tb $kv $(grep -h '^{' "$OUT/f2tb_$kv.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])')" | tee -a "$OUT/session.log"
      done ;;
    x3knobs)  # split-A 64-frame tile / depth knobs after the late staging
      for i in 1 2; do
        for kv in DEF=0 SART_MF_X3_VT=2 SART_MF_X3_DEPTH=3 "SART_MF_X3_VT=2 SART_MF_X3_DEPTH=3" SART_MF_X3_FWD=2,2,as SART_MF_X3_FWD=4,1,as SART_MF_X3_FWD=2,1 SART_MF_X3_FWD=2,2; do
          tag=$(echo "$kv" | tr ' =,' '_-.')
          env $kv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-selfcheck --frames 64 > "$OUT/x3k_${tag}_$i.log" 2>&1 || { echo "FATAL $kv"; exit 1; }
          echo "=== x3k $tag $i $(grep -h '^{' "$OUT/x3k_${tag}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])')" | tee -a "$OUT/session.log"
        done
      done ;;
    bf16w)  # bf16-stored shards at several widths (65536 rows)
      for v in ${BW_LIST:-65536 73728 100000 131072 150000 200000 262144}; do
        timeout -k 10 200 python bench.py --steps 3 --warmup 1 --iters 50 --nvox $v --rtm-dtype bf16 --no-selfcheck > "$OUT/bw_$v.log" 2>&1 || { echo "FATAL $v"; tail -n 20 "$OUT/bw_$v.log"; exit 1; }
        grep -h '^{' "$OUT/bw_$v.log" >> "$OUT/bf16_widths.jsonl"
        echo "=== bf16w $v $(grep -h '^{' "$OUT/bw_$v.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], d["fused_grid"], d["fused_rows_per_tile"])')" | tee -a "$OUT/session.log"
      done ;;
    abbf16kw)  # wide bf16 tiles with kw 5-7 (default) vs kw 8 only (SART_BF16_KW=8)
      run pytest_bf16kw 900 python -u -m pytest tests/test_gpu_bf16.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
      run fcheck_bf16kw 300 python tools/fused_check.py --dtype bf16 8192x150000 16384x100000 8192x200000 65536x163840 &&
      for i in 1 2; do
        for v in 150000 100000 200000 70000 163840 98304; do
          timeout -k 10 200 python bench.py --steps 3 --warmup 1 --iters 50 --nvox $v --rtm-dtype bf16 --no-selfcheck > "$OUT/bk_new_${v}_$i.log" 2>&1 &&
          SART_BF16_KW=8 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --iters 50 --nvox $v --rtm-dtype bf16 --no-selfcheck > "$OUT/bk_old_${v}_$i.log" 2>&1 || { echo "FATAL $v"; exit 1; }
          echo "=== bf16kw $v $i new $(grep -h '^{' "$OUT/bk_new_${v}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], d["fused_grid"], d["fused_rows_per_tile"])') kw8 $(grep -h '^{' "$OUT/bk_old_${v}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], d["fused_grid"], d["fused_rows_per_tile"])')" | tee -a "$OUT/session.log"
        done
      done ;;
    abbf16f4)  # 16-byte flag reads for wide bf16 T = 2 slabs of kw 5-7 (new) vs the one-by-one polls (.abold)
      run pytest_bf16f4 600 python -u -m pytest tests/test_gpu_bf16.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread &&
      for i in 1 2; do
        for v in 150000 163840 200000 70000 262144; do
          timeout -k 10 200 python .abold/bench.py --steps 3 --warmup 1 --iters 50 --nvox $v --rtm-dtype bf16 --no-selfcheck > "$OUT/bf4_old_${v}_$i.log" 2>&1 &&
          timeout -k 10 200 python bench.py --steps 3 --warmup 1 --iters 50 --nvox $v --rtm-dtype bf16 --no-selfcheck > "$OUT/bf4_new_${v}_$i.log" 2>&1 || { echo "FATAL $v"; exit 1; }
          echo "=== bf16f4 $v $i old $(grep -h '^{' "$OUT/bf4_old_${v}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])') new $(grep -h '^{' "$OUT/bf4_new_${v}_$i.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], d["fused_grid"])')" | tee -a "$OUT/session.log"
        done
      done ;;
    benchcols) run bench_cols 600 python bench.py --steps 3 --warmup 1 --partition cols ;;
    benchbf16) run bench_bf16 600 python bench.py --steps 5 --warmup 1 --rtm-dtype bf16 &&
               run bench_bf16_log 600 python bench.py --steps 5 --warmup 1 --rtm-dtype bf16 --variant log ;;
    benchbf16n) SART_BF16_WIDE=0 run bench_bf16_narrow 600 python bench.py --steps 5 --warmup 1 --rtm-dtype bf16 ;;
    benchbf16t) for t in 1 2 4; do
                  SART_FUSED_T=$t run bench_bf16_T$t 300 python bench.py --steps 5 --warmup 1 --rtm-dtype bf16 || exit 1
                done ;;
    benchbf16big) run bench_bf16_512kx256k 900 python bench.py --steps 2 --warmup 1 --rtm-dtype bf16 \
                    --npix 524288 --nvox 262144 --iters 20 ;;
    benchbf16big5) SART_FUSED_SCHEDULE=5 run bench_bf16_512kx256k_s5 900 python bench.py --steps 2 --warmup 1 \
                     --rtm-dtype bf16 --npix 524288 --nvox 262144 --iters 20 ;;
    benchlap) run bench_lap 600 python bench.py --steps 5 --warmup 1 --laplacian ;;
    probe) run probe 600 python tools/probe.py ;;
    ablation) run ablation_bf16 600 python tools/fused_ablation.py --dtype bf16 65536x262144 65536x65536 &&
              run ablation_fp32 600 python tools/fused_ablation.py --dtype fp32 65536x262144 65536x65536 65536x100000 ;;
    sched7) SEL="tests/test_gpu_bf16.py tests/test_gpu_solver.py" run pytest_sched7 900 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_solver.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread &&
            run ablation_s7 600 python tools/fused_ablation.py --dtype bf16 65536x262144 &&
            SART_BF16_T2_SCHED=6 run ablation_s6 600 python tools/fused_ablation.py --dtype bf16 65536x262144 &&
            run fcheck_s7 600 python tools/fused_check.py --dtype bf16 8192x262144 65536x262144 ;;
    prefetch) run pytest_prefetch 900 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_solver.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread &&
              run ablation_pf_fp32 600 python tools/fused_ablation.py --dtype fp32 65536x100000 65536x200000 65536x70000 65536x262144 65536x65536 &&
              run ablation_pf_bf16 600 python tools/fused_ablation.py --dtype bf16 65536x262144 65536x65536 65536x100000 &&
              run fcheck_pf 600 python tools/fused_check.py 8192x100000 8192x200000 65536x262144 16384x65536 &&
              run bench_pf 600 python bench.py --steps 5 --warmup 1 ;;
    ab) for i in 1 2; do
          run ab_new_$i 300 python tools/fused_ablation.py --dtype fp32 ${AB_SHAPES:-65536x100000 65536x200000 65536x262144 65536x65536} &&
          run ab_old_$i 300 python .abold/tools/fused_ablation.py --dtype fp32 ${AB_SHAPES:-65536x100000 65536x200000 65536x262144 65536x65536} || exit 1
        done ;;
    abtests) run pytest_ab 900 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_solver.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread &&
             run fcheck_ab 600 python tools/fused_check.py 8192x100000 8192x200000 65536x262144 16384x65536 &&
             run fcheck_ab_bf16 600 python tools/fused_check.py --dtype bf16 65536x262144 16384x65536 ;;
    abbf16) for i in 1 2; do
              run abb_new_$i 300 python tools/fused_ablation.py --dtype bf16 65536x262144 65536x65536 65536x100000 &&
              run abb_old_$i 300 python .abold/tools/fused_ablation.py --dtype bf16 65536x262144 65536x65536 65536x100000 || exit 1
            done ;;
    abdpp) for x in 0 16 32 48; do
             SART_FUSED_DBG_EXTRA=$x run abdpp_$x 300 python tools/fused_ablation.py --dtype fp32 65536x200000 65536x100000 65536x70000 || exit 1
           done ;;
    abdpp2) for x in 0 16 32 48; do
             SART_FUSED_DBG_EXTRA=$x run abdpp2_$x 300 python tools/fused_ablation.py --dtype bf16 65536x262144 65536x65536 65536x100000 &&
             SART_FUSED_DBG_EXTRA=$x run abdpp3_$x 300 python tools/fused_ablation.py --dtype fp32 65536x65536 65536x262144 65536x200000 || exit 1
           done ;;
    abmf) run pytest_mf 900 python -u -m pytest tests/test_gpu_multiframe.py tests/test_gpu_multiframe_bf16.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread &&
          run x3acc 300 python tools/x3_accuracy.py &&
          for i in 1 2; do
            run abmf_new64_$i 300 python bench.py --steps 3 --warmup 1 --frames 64 &&
            run abmf_old64_$i 300 python .abold/bench.py --steps 3 --warmup 1 --frames 64 &&
            run abmf_new32_$i 300 python bench.py --steps 3 --warmup 1 --frames 32 &&
            run abmf_old32_$i 300 python .abold/bench.py --steps 3 --warmup 1 --frames 32 || exit 1
          done ;;
    abmf2) for i in 1 2; do
            run abmf2_new64_$i 300 python bench.py --steps 3 --warmup 1 --frames 64 &&
            run abmf2_old64_$i 300 python .abold/bench.py --steps 3 --warmup 1 --frames 64 &&
            run abmf2_new32_$i 300 python bench.py --steps 3 --warmup 1 --frames 32 &&
            run abmf2_old32_$i 300 python .abold/bench.py --steps 3 --warmup 1 --frames 32 || exit 1
          done && run x3acc2 300 python tools/x3_accuracy.py ;;
    abmfb) run pytest_mfb 900 python -u -m pytest tests/test_gpu_multiframe.py tests/test_gpu_multiframe_bf16.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread &&
           for i in 1 2; do
             for spec in "b64|--frames 64 --rtm-dtype bf16" "f64|--frames 64" "b32|--frames 32 --rtm-dtype bf16" "f32|--frames 32"; do
               name=${spec%%|*}; args=${spec#*|}
               run abmfb_new_${name}_$i 300 python bench.py --steps 3 --warmup 1 --no-selfcheck $args &&
               run abmfb_old_${name}_$i 300 python .abold/bench.py --steps 3 --warmup 1 --no-selfcheck $args || exit 1
             done
           done ;;
    mfblocks) for kv in DEF=0 SART_MF_FWD_BLOCKS=768 SART_MF_FWD_BLOCKS=1536 SART_MF_FWD_BLOCKS=2048 SART_MF_FWD_BLOCKS=3072 \
                      SART_MF_BP_BLOCKS=768 SART_MF_BP_BLOCKS=1536 SART_MF_BP_BLOCKS=2048 SART_MF_BP_BLOCKS=3072 DEF=1; do
                for spec in "b64|--frames 64 --rtm-dtype bf16" "f64|--frames 64"; do
                  name=${spec%%|*}; args=${spec#*|}
                  env "$kv" timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-selfcheck $args > "$OUT/mfblk_${name}_$kv.log" 2>&1 || { echo "FATAL $kv"; exit 1; }
                  echo "=== mfblk $name $kv $(grep -h '^{' "$OUT/mfblk_${name}_$kv.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])')" | tee -a "$OUT/session.log"
                done
              done ;;
    pmcmfb) echo "=== pmcmfb" >> "$OUT/session.log"
           timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
             -d "$OUT/pmc_mfb64" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames 64 --iters 5 --npix 16384 --rtm-dtype bf16 --no-selfcheck > "$OUT/pmc_mfb64.log" 2>&1
           rc=$?; echo "=== pmcmfb rc=$rc" >> "$OUT/session.log"; tail -5 "$OUT/pmc_mfb64.log"; [ $rc -eq 0 ] || exit $rc
           timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE \
             -d "$OUT/pmc_mfb64_insts" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames 64 --iters 5 --npix 16384 --rtm-dtype bf16 --no-selfcheck > "$OUT/pmc_mfb64_insts.log" 2>&1
           rc=$?; echo "=== pmcmfb insts rc=$rc" >> "$OUT/session.log"; [ $rc -eq 0 ] || exit $rc ;;
    pmcmf) echo "=== pmcmf" >> "$OUT/session.log"
           timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
             -d "$OUT/pmc_mf64" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames 64 --iters 5 --npix 16384 --no-selfcheck > "$OUT/pmc_mf64.log" 2>&1
           rc=$?; echo "=== pmcmf rc=$rc" >> "$OUT/session.log"; tail -5 "$OUT/pmc_mf64.log"; [ $rc -eq 0 ] || exit $rc ;;
    abpreset) for i in 1 2; do
            run abp_new_$i 300 python bench.py --config 512kx256k --steps 3 --warmup 1 --no-selfcheck &&
            run abp_old_$i 300 python .abold/bench.py --config 512kx256k --steps 3 --warmup 1 --no-selfcheck || exit 1
          done ;;
    abgraph) for i in 1 2; do
            run abg_def_$i 300 python bench.py --steps 5 --warmup 1 --no-selfcheck &&
            SART_GRAPH=1 run abg_graph_$i 300 python bench.py --steps 5 --warmup 1 --no-selfcheck || exit 1
          done ;;
    testsrest) run pytest_gpu_rest 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    rehearse8) SART_DIST_BACKEND=gloo SART_P2P=1 SART_P2P_TIMEOUT_S=60 run comm_check_p2p_n8 300 python -m torch.distributed.run --nnodes=1 \
                 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29608 tools/comm_check.py --out "$OUT/comm_check_p2p_n8.json" &&
               SART_P2P=1 SART_P2P_TIMEOUT_S=60 run bench_share8_p2p 400 python bench.py --gpus 8 --share-gpus --npix 4096 --steps 2 --warmup 1 --iters 20 --watchdog 200 ;;
    mf16sweep) run rocprof_mf16 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_mf16" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames 16 --iters 20 &&
               for kv in DEF=0 SART_MF_DEPTH=1 SART_MF_DEPTH=2 SART_MF_DEPTH=3 SART_MF_ROWS=2 SART_MF_VOX=2 SART_MF_NT=1 SART_MF_BP_BLOCKS=1024 SART_MF_BP_BLOCKS=256 DEF=1; do
                 env "$kv" timeout -k 10 300 python bench.py --steps 2 --warmup 1 --frames 16 --iters 50 > "$OUT/mf16_$kv.log" 2>&1 || { echo "FATAL $kv"; exit 1; }
                 echo "=== mf16 $kv $(grep -h '^{' "$OUT/mf16_$kv.log" | python -c 'import sys,json; print(json.loads(sys.stdin.readline())["iters_per_s"])')" | tee -a "$OUT/session.log"
               done ;;
    mf16x3) for i in 1 2; do
              run mf16_x3on_$i 300 python bench.py --steps 2 --warmup 1 --frames 16 --iters 50 --mf-split-a on &&
              run mf16_x3off_$i 300 python bench.py --steps 2 --warmup 1 --frames 16 --iters 50 --mf-split-a off || exit 1
            done &&
            run rocprof_mf16x3 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_mf16x3" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames 16 --iters 20 --mf-split-a on ;;
    mf16as) for kv in SART_MF_X3_FWD=2,2 SART_MF_X3_FWD=2,2,as SART_MF_X3_FWD=2,1,as SART_MF_X3_FWD=4,1,as SART_MF_X3_FWD=4,2,as SART_MF_X3_FWD=4,1 SART_MF_X3_DEPTH=2; do
              env "$kv" timeout -k 10 300 python bench.py --steps 2 --warmup 1 --frames 16 --iters 50 --mf-split-a on > "$OUT/mf16as_$kv.log" 2>&1 || { echo "FATAL $kv"; exit 1; }
              echo "=== mf16as $kv $(grep -h '^{' "$OUT/mf16as_$kv.log" | python -c 'import sys,json; print(json.loads(sys.stdin.readline())["iters_per_s"])')" | tee -a "$OUT/session.log"
            done ;;
    finalmatrix) for spec in "default|" "log|--variant log" "lap|--laplacian" "twopass|--no-fused" "cols|--partition cols" "bf16|--rtm-dtype bf16" "bf16log|--rtm-dtype bf16 --variant log" "mf16|--frames 16" "mf32|--frames 32" "mf64|--frames 64" "mfb16|--frames 16 --rtm-dtype bf16" "mfb32|--frames 32 --rtm-dtype bf16" "mfb64|--frames 64 --rtm-dtype bf16"; do
                   name=${spec%%|*}; args=${spec#*|}
                   timeout -k 10 300 python bench.py --steps 3 --warmup 1 $args > "$OUT/final_$name.log" 2>&1 || { echo "FATAL $name"; exit 1; }
                   echo "=== final $name $(grep -h '^{' "$OUT/final_$name.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])')" | tee -a "$OUT/session.log"
                 done ;;
    abkw8) for i in 1 2; do
            run abk_new_$i 300 python bench.py --config 512kx256k --steps 3 --warmup 1 --no-selfcheck &&
            run abk_old_$i 300 python .abold/bench.py --config 512kx256k --steps 3 --warmup 1 --no-selfcheck || exit 1
          done &&
          run abk_fc 300 python tools/fused_check.py 65536x262144 ;;
    abt4) for i in 1 2; do
            run abt4_new_$i 300 python bench.py --steps 5 --warmup 1 --no-selfcheck &&
            run abt4_old_$i 300 python .abold/bench.py --steps 5 --warmup 1 --no-selfcheck || exit 1
          done ;;
    abbf) for i in 1 2; do
            run abbf_dpp_$i 300 python bench.py --steps 5 --warmup 1 --rtm-dtype bf16 --no-selfcheck &&
            run abbf_shfl_$i 300 python .abold/bench.py --steps 5 --warmup 1 --rtm-dtype bf16 --no-selfcheck || exit 1
          done &&
          run abbfbig_dpp 600 python bench.py --steps 2 --warmup 1 --rtm-dtype bf16 --npix 524288 --nvox 262144 --iters 20 --no-selfcheck &&
          run abbfbig_shfl 600 python .abold/bench.py --steps 2 --warmup 1 --rtm-dtype bf16 --npix 524288 --nvox 262144 --iters 20 --no-selfcheck ;;
    bf16final) run pytest_bf16f 900 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_solver.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread &&
               run bench_bf16f 300 python bench.py --steps 5 --warmup 1 --rtm-dtype bf16 &&
               run bench_bf16bigf 600 python bench.py --steps 2 --warmup 1 --rtm-dtype bf16 --npix 524288 --nvox 262144 --iters 20 &&
               run bench_f 300 python bench.py --steps 5 --warmup 1 ;;
    probemall) run probe_mall 600 python tools/probe_mall.py ;;
    fcheck) run fcheck_bf16 600 python tools/fused_check.py --dtype bf16 8192x262144 65536x262144 &&
            SART_FUSED_SCHEDULE=5 run fcheck_bf16_s5 600 python tools/fused_check.py --dtype bf16 65536x262144 &&
            run fcheck_fp32 600 python tools/fused_check.py 8192x262144 65536x262144 16384x65536 ;;
    foldsmall) SART_FUSED_FOLD=0 run fcheck_small_nofold 150 python tools/fused_check.py 16384x262144 &&
              run fcheck_small_fold 150 python tools/fused_check.py 16384x262144 &&
              SART_FUSED_FOLD=8 run fcheck_small_fold8 150 python tools/fused_check.py --dtype bf16 8192x131072 ;;
    foldperf) for v in 200000 100000 262144; do
                run bench_w${v}_fold 300 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck &&
                SART_FUSED_FOLD=0 run bench_w${v}_nofold 300 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck || exit 1
              done ;;
    foldcheck) run fcheck_fold_bf16 600 python tools/fused_check.py --dtype bf16 65536x262144 &&
              SART_FUSED_FOLD=0 run fcheck_nofold_bf16 600 python tools/fused_check.py --dtype bf16 65536x262144 &&
              SART_FUSED_FOLD=64 run fcheck_fold64_bf16 600 python tools/fused_check.py --dtype bf16 65536x262144 &&
              run fcheck_fold_fp32 600 python tools/fused_check.py 65536x262144 8192x204800 &&
              run bench_w200000 300 python bench.py --steps 3 --warmup 1 --nvox 200000 &&
              SART_FUSED_FOLD=0 run bench_w200000_nofold 300 python bench.py --steps 3 --warmup 1 --nvox 200000 ;;
    numerics) run numerics 600 python tools/numerics_check.py ;;
    kwcheck) run fcheck_kw 600 python tools/fused_check.py 8192x70000 8192x100000 8192x150000 8192x200000 4096x229376 ;;
    benchw) for v in 65536 60000 100000 200000 70000 150000; do
              run bench_w$v 300 python bench.py --steps 3 --warmup 1 --nvox $v --no-selfcheck || exit 1
            done ;;
    trace) run fused_trace 600 python tools/fused_trace.py ;;
    probef) PROBE_FUSED_ONLY=1 run probe_fused 600 python tools/probe.py ;;
    probet1) PROBE_FUSED_ONLY=1 PROBE_CFGS=6:1:0,6:1:5,6:0:4 run probe_t1 600 python tools/probe.py \
              4096x262144 4096x204800 16384x73728 8192x106496 16384x65536 8192x131072 ;;
    probew) PROBE_FUSED_ONLY=1 PROBE_CFGS=${PROBE_CFGS:-6:0:4,3:0:0} run probe_widths 600 python tools/probe.py \
              16384x65536 16384x61440 16384x73728 8192x131072 8192x102400 4096x262144 4096x204800 ;;
    commcheck) for n in 2 4; do
                 SART_DIST_BACKEND=gloo SART_P2P=1 run comm_check_p2p_n$n 300 python -m torch.distributed.run --nnodes=1 \
                   --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) tools/comm_check.py \
                   --out "$OUT/comm_check_p2p_n$n.json" || exit 1
               done ;;
    testsel) run pytest_sel 900 python -u -m pytest ${SEL:-tests} -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    profbf16) run rocprof_bf16 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bf16" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --rtm-dtype bf16 &&
              run rocprof_bf16_pmc 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/prof_bf16_pmc" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 20 --rtm-dtype bf16 ;;
    profr2) run rocprof_r2_fp32 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r2_fp32" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 &&
            run rocprof_r2_bf16_big 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r2_bf16_big" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --rtm-dtype bf16 --npix 524288 --nvox 262144 --iters 20 &&
            run rocprof_r2_mfb64 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r2_mfb64" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames 64 --iters 20 --rtm-dtype bf16 ;;
    prof) run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 ;;
    r4info)  # scheduler limits that decide whether N processes' queues are all resident (no GPU work)
      { echo "hws_max_conc_proc: $(cat /sys/module/amdgpu/parameters/hws_max_conc_proc 2>&1)";
        echo "sched_policy: $(cat /sys/module/amdgpu/parameters/sched_policy 2>&1)";
        echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}";
        for d in /sys/class/kfd/kfd/topology/nodes/*; do
          if grep -q "simd_count [1-9]" "$d/properties" 2>/dev/null; then
            grep -E "num_cp_queues|num_sdma|simd_count|cu_per_simd|max_waves_per_simd|num_xcc|array_count|max_slots" "$d/properties"; fi
        done; } > "$OUT/r4info.txt" 2>&1; cat "$OUT/r4info.txt" ;;
    r4comm)  # P2P all-reduce at 4 and 8 processes on one GPU (forced p2p, gloo host side): bitwise + set-up time
      for n in 4 8; do
        SART_DIST_BACKEND=gloo SART_P2P=1 run comm_check_p2p_n$n 300 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29610 + n)) tools/comm_check.py \
          --out "$OUT/comm_check_p2p_n$n.json" || exit 1
        python -c "import json; d=json.load(open('$OUT/comm_check_p2p_n$n.json')); print('n$n', d['backend'], d['setup_s'], d['us_per_call'], all(r['exact'] or r['n']*4>2**21 for r in d['results'])); print(d['describe'])" | tee -a "$OUT/session.log"
      done ;;
    r4reh8)  # 8-rank one-GPU rehearsal of bench --gpus 8 (fused sweep per rank on 32 CUs + P2P auto vs staged)
      run bench_share8_r4 300 python bench.py --gpus 8 --share-gpus --npix 16384 --steps 3 --warmup 1 --watchdog 300 ;;
    r4reh8q1)  # the same with one hardware queue per process (8 queues in all: no queue over-subscription)
      GPU_MAX_HW_QUEUES=1 run bench_share8_r4_q1 300 python bench.py --gpus 8 --share-gpus --npix 16384 --steps 3 --warmup 1 --watchdog 300 ;;
    r4reh4) run bench_share4_r4 500 python bench.py --gpus 4 --share-gpus --npix 32768 --steps 3 --warmup 1 --watchdog 300 ;;
    r4load) run load_bench 900 python tools/load_bench.py ;;
    r4abl) run probe_abl 300 python tools/probe_mf_abl.py &&
           run probe_abl_2tb 300 python tools/probe_mf_abl.py 16384x262144 ;;
    r4strong)  # strong scaling of the 64k x 64k headline over ranks sharing one GPU: 32768 / 16384 / 8192 rows per rank
      for n in 2 4 8; do
        timeout -k 10 300 python bench.py --gpus $n --share-gpus --scaling strong --steps 3 --warmup 1 --watchdog 240 \
          > "$OUT/strong_n$n.log" 2>&1 || { echo "FATAL strong $n"; tail -n 30 "$OUT/strong_n$n.log"; exit 1; }
        grep -h '^{' "$OUT/strong_n$n.log" >> "$OUT/strong.jsonl"
        echo "=== strong n$n $(grep -h '^{' "$OUT/strong_n$n.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["allreduce_us_per_iter"], d["allreduce"][:60], d["allreduce_fallbacks"], d["fused_grid"])')" | tee -a "$OUT/session.log"
      done ;;
    r4cw)  # chip-wide row groups: per-CU rate by slab width kw (forced) at widths > 294912 (J must divide the width)
      for spec in ${CW_SPECS:-8:303104 8:311296 8:327680 8:344064 7:301056 7:308224 7:315392 6:307200 6:313344 6:325632 9:304128 9:313344 9:331776 5:307200 5:327680}; do
        k=${spec%%:*}; v=${spec#*:}
        SART_FUSED_KW=$k timeout -k 10 200 python bench.py --steps 3 --warmup 1 --iters 50 --nvox $v --ld $v --npix 32768 --no-selfcheck \
          > "$OUT/cw_${k}_$v.log" 2>&1 || { echo "FATAL $spec"; tail -n 20 "$OUT/cw_${k}_$v.log"; exit 1; }
        grep -h '^{' "$OUT/cw_${k}_$v.log" >> "$OUT/cw_kw.jsonl"
        echo "=== cw kw$k $v $(grep -h '^{' "$OUT/cw_${k}_$v.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); g=d["fused_grid"]; print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], g, d["fused_schedule"], round(d["effective_hbm_TBps_per_gpu"]*1e3/g["workgroups"], 2), "GB/s/CU")')" | tee -a "$OUT/session.log"
      done ;;
    r4cwsweep)  # default geometry at 294912 ... 557056 voxels in steps of 8192 (chip-wide row groups above 294912)
      : > "$OUT/cw_sweep.jsonl"
      for v in $(seq ${CWS_FROM:-294912} 8192 ${CWS_TO:-557056}) ${CWS_EXTRA:-}; do
        timeout -k 10 200 python bench.py --steps 3 --warmup 1 --iters 50 --nvox $v --npix 32768 --no-selfcheck \
          > "$OUT/cws_$v.log" 2>&1 || { echo "FATAL $v"; tail -n 20 "$OUT/cws_$v.log"; exit 1; }
        grep -h '^{' "$OUT/cws_$v.log" >> "$OUT/cw_sweep.jsonl"
        echo "=== cws $v $(grep -h '^{' "$OUT/cws_$v.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); g=d["fused_grid"]; print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], g["ld"], g["kw"], g["J"], g["I"], g["xcd_local"], d["fused_schedule"])')" | tee -a "$OUT/session.log"
        rm -f "$OUT/cws_$v.log"
      done ;;
    r4xblk) run probe_xblk 400 python tools/probe_mf_xblk.py ;;
    r4mftest) run pytest_mf 600 python -u -m pytest tests/test_gpu_multiframe_bf16.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "blocked or split_a or vs_oracle" ;;
    r4cwtest) run pytest_cw 600 python -u -m pytest tests/test_gpu_solver.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "production_geometry or chip_wide" ;;
    r4cwab)  # A/B of chip-wide settings: for each width, every "NAME=VAL[,NAME=VAL]" setting of CWAB_SETS (":" = defaults)
      : > "$OUT/cw_ab.jsonl"
      for v in ${CWAB_WIDTHS:-303104 327680 360448 393216 450560 458752 524288 557056}; do
        for set in ${CWAB_SETS:-: SART_FUSED_GPAD=0}; do
          envs=(); [ "$set" != ":" ] && IFS=, read -ra envs <<< "$set"
          env "${envs[@]}" timeout -k 10 200 python bench.py --steps 3 --warmup 1 --iters 50 --nvox $v --npix 32768 ${CWAB_ARGS:---no-selfcheck} \
            > "$OUT/cwab.log" 2>&1 || { echo "FATAL $v $set"; tail -n 20 "$OUT/cwab.log"; exit 1; }
          grep -h '^{' "$OUT/cwab.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); d["ab_set"]=sys.argv[1]; print(json.dumps(d))' "$set" >> "$OUT/cw_ab.jsonl"
          echo "=== cwab $v $set $(tail -n 1 "$OUT/cw_ab.jsonl" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); g=d["fused_grid"]; print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"], g["ld"], g["kw"], g["J"], g["I"], g["xcd_local"], d["fused_schedule"])')" | tee -a "$OUT/session.log"
        done
      done ;;
    r4mf) run bench_mfx64_blk 600 python bench.py --steps 3 --warmup 1 --frames 64 &&
          SART_MF_XBLK=0 run bench_mfx64_fm 600 python bench.py --steps 3 --warmup 1 --frames 64 &&
          run bench_mfb64_blk 600 python bench.py --steps 3 --warmup 1 --frames 64 --rtm-dtype bf16 &&
          run bench_2tb_blk 900 python bench.py --config 2tb --steps 2 --warmup 1 ;;
    r4tiles) PROBE_STORAGE=fp32 PROBE_TILES="2,1,as:3;2,1,as:2;4,1,as:3;4,1,as:2;2,2,as:2;2,2,as:3;4,1:3;2,2:2;4,2,as:2" \
               run probe_tiles 600 python tools/probe_mf_xblk.py ;;
    r4lastbwd)  # final-sweep back-projection skipped (default) vs run (SART_MF_LAST_BWD=1)
              run pytest_mf 600 python -u -m pytest tests/test_gpu_multiframe.py tests/test_gpu_multiframe_bf16.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider &&
              run bench_2tb_skip 600 python bench.py --config 2tb --steps 2 --warmup 1 &&
              SART_MF_LAST_BWD=1 run bench_2tb_full 600 python bench.py --config 2tb --steps 2 --warmup 1 &&
              run bench_mfx64_skip 300 python bench.py --steps 3 --warmup 1 --frames 64 &&
              run bench_mfb64_skip 300 python bench.py --steps 3 --warmup 1 --frames 64 --rtm-dtype bf16 ;;
    r4mf128)  # 128-frame split-A batches: kernels + engine tests, then 64 / 128-frame benches
              run pytest_mf128 600 python -u -m pytest tests/test_gpu_multiframe_bf16.py -k "128" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider &&
              run pytest_mf 900 python -u -m pytest tests/test_gpu_multiframe.py tests/test_gpu_multiframe_bf16.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider &&
              run bench_mfx64 300 python bench.py --steps 3 --warmup 1 --frames 64 &&
              run bench_mfx128 300 python bench.py --steps 3 --warmup 1 --frames 128 &&
              run bench_mfb64 300 python bench.py --steps 3 --warmup 1 --frames 64 --rtm-dtype bf16 &&
              run rocprof_mfx128 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_mfx128" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames 128 --iters 20 --no-selfcheck ;;
    r4mfb128)  # 128-frame bf16-storage batches: tests, bench, kernel trace
              run pytest_mfb128 600 python -u -m pytest tests/test_gpu_multiframe_bf16.py -k "128" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider &&
              run bench_mfb128 300 python bench.py --steps 3 --warmup 1 --frames 128 --rtm-dtype bf16 &&
              run rocprof_mfb128 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_mfb128" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames 128 --iters 20 --rtm-dtype bf16 --no-selfcheck ;;
    r4tbab)  # 2tb preset (64 frames) A/B over env settings (MFAB_SETS as r4mfab)
      : > "$OUT/tb_ab.jsonl"
      for set in ${MFAB_SETS:-: SART_MF_X3_FWD=2,1,as SART_MF_FWD_BLOCKS=512 SART_MF_FWD_BLOCKS=2048}; do
        envs=(); [ "$set" != ":" ] && IFS=+ read -ra envs <<< "$set"
        env "${envs[@]}" timeout -k 10 400 python bench.py --config 2tb --steps 2 --warmup 1 > "$OUT/tbab.log" 2>&1 \
          || { echo "FATAL $set"; tail -n 20 "$OUT/tbab.log"; exit 1; }
        grep -h '^{' "$OUT/tbab.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); d["ab_set"]=sys.argv[1]; print(json.dumps(d))' "$set" >> "$OUT/tb_ab.jsonl"
        echo "=== tbab $set $(tail -n 1 "$OUT/tb_ab.jsonl" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])')" | tee -a "$OUT/session.log"
      done ;;
    r4mffinal)  # multi-frame suites and the 64 / 128-frame benches of both storages
              run pytest_mf 900 python -u -m pytest tests/test_gpu_multiframe.py tests/test_gpu_multiframe_bf16.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider &&
              for a in "--frames 64" "--frames 128" "--frames 64 --rtm-dtype bf16" "--frames 128 --rtm-dtype bf16"; do
                run bench_mf 300 python bench.py --steps 3 --warmup 1 $a || exit 1
                grep -h '^{' "$OUT/bench_mf.log" >> "$OUT/mf_final.jsonl"
              done ;;
    r4prof2tb) run rocprof_2tb 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_2tb" -o run --output-format csv -- python3 bench.py --config 2tb --steps 1 --warmup 0 --no-selfcheck &&
               run rocprof_mfb64 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_mfb64" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames 64 --iters 20 --rtm-dtype bf16 --no-selfcheck ;;
    r4profmf) run rocprof_mfx64 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_mfx64" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --frames 64 --iters 20 --no-selfcheck ;;
    r4m32) PROBE_ABL=0 PROBE_BWD="${M32_SET:-lds:2,h16:2,lds:2,h16:2}" run probe_m32 300 python tools/probe_mf_abl.py &&
           PROBE_ABL=0 PROBE_BWD="${M32_SET:-lds:2,h16:2,lds:2,h16:2}" run probe_m32_2tb 300 python tools/probe_mf_abl.py 16384x262144 ;;
    r4bf16cw)  # wide bf16 tiles, XCD-local vs chip-wide groups, self-check on (rc 1 = self-check failed: keep going)
      for spec in "131072:1:" "131072:0:" "150000:0:4" "150000:0:2" "163840:0:" "150000:1:"; do
        IFS=: read -r v xl t <<< "$spec"
        SART_BF16_XL=$xl SART_BF16_T=$t run bf16cw_${v}_${xl}_${t} 200 python bench.py --steps 3 --warmup 1 --iters 50 --nvox $v --npix 32768 --rtm-dtype bf16 || exit 1
        grep -h '^{' "$OUT/bf16cw_${v}_${xl}_${t}.log" >> "$OUT/bf16cw.jsonl" || true
        grep -h "self-check" "$OUT/bf16cw_${v}_${xl}_${t}.log" | tail -1 || true
      done ;;
    r4mfab)  # multi-frame A/B over env settings (MFAB_SETS, "+" joins variables; ":" = defaults), 64 frames, both storages
      : > "$OUT/mf_ab.jsonl"
      for args in "--frames 64" "--frames 64 --rtm-dtype bf16" ${MFAB_EXTRA:-}; do
        for set in ${MFAB_SETS:-: SART_MF_WEARLY=0 SART_MF_WEARLY=1 SART_MF_XEARLY=0}; do
          envs=(); [ "$set" != ":" ] && IFS=+ read -ra envs <<< "$set"
          env "${envs[@]}" timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-selfcheck $args > "$OUT/mfab.log" 2>&1 \
            || { echo "FATAL $args $set"; tail -n 20 "$OUT/mfab.log"; exit 1; }
          grep -h '^{' "$OUT/mfab.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); d["ab_set"]=sys.argv[1]; d["ab_args"]=sys.argv[2]; print(json.dumps(d))' "$set" "$args" >> "$OUT/mf_ab.jsonl"
          echo "=== mfab [$args] $set $(tail -n 1 "$OUT/mf_ab.jsonl" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])')" | tee -a "$OUT/session.log"
        done
      done ;;
    r4mf128ab)  # 128-frame split-A A/B over env settings (MFAB_SETS as r4mfab)
      : > "$OUT/mf128_ab.jsonl"
      for set in ${MFAB_SETS:-: SART_MF_X3_FWD=2,2,as SART_MF_X3_DEPTH=3 SART_MF_H16=ew SART_MF_H16=ew+SART_MF_X3_DEPTH=3}; do
        envs=(); [ "$set" != ":" ] && IFS=+ read -ra envs <<< "$set"
        env "${envs[@]}" timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-selfcheck --frames 128 ${MF128_ARGS:-} > "$OUT/mfab.log" 2>&1 \
          || { echo "FATAL $set"; tail -n 20 "$OUT/mfab.log"; exit 1; }
        grep -h '^{' "$OUT/mfab.log" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); d["ab_set"]=sys.argv[1]; print(json.dumps(d))' "$set" >> "$OUT/mf128_ab.jsonl"
        echo "=== mf128ab $set $(tail -n 1 "$OUT/mf128_ab.jsonl" | python -c 'import sys,json; d=json.loads(sys.stdin.readline()); print(d["iters_per_s"], d["effective_hbm_TBps_per_gpu"])')" | tee -a "$OUT/session.log"
      done ;;
    r4bf16seg)  # chip-wide bf16 at 150000 voxels: does a shorter back-projection chain (segments) fix the self-check?
      for seg in 280 700; do
        SART_BF16_XL=0 SART_BF16_T=4 SART_FUSED_SEG=$seg run bf16seg_$seg 200 python bench.py --steps 3 --warmup 1 --iters 50 --nvox 150000 --npix 32768 --rtm-dtype bf16 || true
        grep -h "self-check\|^{" "$OUT/bf16seg_$seg.log" | cut -c1-300 | tail -2 || true
      done
      SART_BF16_XL=1 run bf16seg_xl 200 python bench.py --steps 3 --warmup 1 --iters 50 --nvox 150000 --npix 32768 --rtm-dtype bf16 || true ;;
    r4bf16test) run pytest_bf16 900 python -u -m pytest tests/test_gpu_bf16.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    r4pmcbwd)  # PMC of the split-A 64-frame back-projection (probe, default kernel): issue / co-execution counters
      PROBE_ABL=0 PROBE_BWD="lds:2" timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE \
        -d "$OUT/pmc_bwd" -o run --output-format csv -- python3 tools/probe_mf_abl.py > "$OUT/pmc_bwd.log" 2>&1 || { echo "FATAL pmc"; tail -n 20 "$OUT/pmc_bwd.log"; exit 1; } ;;
    r4cli) run pytest_cli 900 python -u -m pytest tests/test_native_driver.py tests/test_cli_e2e.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    r4bench) run bench_r4 300 python bench.py --steps 20 --warmup 5 ;;
    r4dist) run pytest_dist 1100 python -u -m pytest tests/test_gpu_distributed.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    r5share)  # the round driver's launch (torchrun, one process per rank) rehearsed on ONE GPU: 2 and 8 ranks share it
      for n in 2 8; do
        run bench_share${n}_torchrun_r5 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
          --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --share-gpus --steps 3 --warmup 1 \
          --watchdog 300 || exit 1
        grep -h '^{' "$OUT/bench_share${n}_torchrun_r5.log" > "$OUT/bench_share${n}_torchrun_r5.json" || true
      done ;;
    pmcfinal)  # HBM bytes (FETCH_SIZE) and occupancy counters of the headline fused sweep, the sparse kernels and the
               # 64-frame split-A kernels, each pass its own run with the kernel trace (durations) beside the counters
      PMC_OCC="SQ_WAVES SQ_LEVEL_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
      for spec in "head|bench.py --steps 1 --warmup 0 --no-selfcheck" \
                  "sparse|tools/sparse_bench.py --no-dense --steps 1 --iters 20 --frames 64" \
                  "mf64|bench.py --steps 1 --warmup 0 --frames 64 --iters 5 --no-selfcheck"; do
        tag=${spec%%|*}; cmd=${spec#*|}
        for pass in fetch occ; do
          if [ $pass = fetch ]; then ctr="FETCH_SIZE GRBM_GUI_ACTIVE"; else ctr=$PMC_OCC; fi
          echo "=== pmc_${tag}_$pass ($(date +%T))" | tee -a "$OUT/session.log"
          timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d "$OUT/pmc_${tag}_$pass" -o run --output-format csv \
            -- python3 $cmd > "$OUT/pmc_${tag}_$pass.log" 2>&1
          rc=$?; echo "=== pmc_${tag}_$pass rc=$rc" | tee -a "$OUT/session.log"; tail -n 3 "$OUT/pmc_${tag}_$pass.log"
          case $rc in 0|1) ;; *) echo "FATAL pmc rc=$rc" | tee -a "$OUT/session.log"; exit $rc ;; esac
        done
      done
      python3 tools/pmc_summary.py "$OUT"/pmc_head_* "$OUT"/pmc_sparse_* "$OUT"/pmc_mf64_* > "$OUT/pmc_summary.txt" 2>&1 || true ;;
    r6tail)  # the N > 1 single-frame iteration tail (collective + decide / update) at strong-scaling
             # shard sizes, 2 / 4 / 8 ranks sharing one GPU, the P2P kernel with and without the fused update
      for npix in ${TAIL_NPIX:-8192 16384}; do
        for n in ${TAIL_N:-2 4 8}; do
          for fu in 1 0; do
            name=tail_np${npix}_n${n}_fu$fu
            SART_P2P_FUSED_UPDATE=$fu run $name 300 python bench.py --gpus $n --share-gpus --npix $npix --steps 3 \
              --warmup 1 --watchdog 240 --no-selfcheck || exit 1
            grep -h '^{' "$OUT/$name.log" | python3 -c "import sys,json; d=json.loads(sys.stdin.readline()); d['tag']='$name'; d['fused_update']=$fu; print(json.dumps(d))" >> "$OUT/tail_r6.jsonl" || exit 1
          done
        done
      done ;;
    r6tailprof)  # kernel trace of the same runs, fused update on / off: every rank started here under its own
                 # rocprofv3 (the program itself after --, no launcher hop), the --share-gpus environment set by hand
      for n in ${TAIL_N:-2 8}; do
        q=$(( 12 / n )); [ $q -lt 1 ] && q=1; [ $q -gt 4 ] && q=4
        for fu in 1 0; do
          name=tailprof_np8192_n${n}_fu$fu
          echo "=== $name ($(date +%T))" | tee -a "$OUT/session.log"
          port=$(( 29700 + n * 2 + fu ))
          pids=""
          for r in $(seq 0 $((n - 1))); do
            SART_P2P_FUSED_UPDATE=$fu RANK=$r LOCAL_RANK=$r WORLD_SIZE=$n LOCAL_WORLD_SIZE=$n MASTER_ADDR=127.0.0.1 \
              MASTER_PORT=$port SART_DIST_BACKEND=gloo SART_P2P_WRAP_STAGED=1 SART_FUSED_SHARED=1 GPU_MAX_HW_QUEUES=$q \
              timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/$name/r$r" -o run -- \
              python3 bench.py --gpus $n --share-gpus --npix 8192 --steps 2 --warmup 1 --watchdog 240 --no-selfcheck \
              > "$OUT/${name}_r$r.log" 2>&1 &
            pids="$pids $!"
          done
          rc=0
          for p in $pids; do wait $p || rc=$?; done
          echo "=== $name rc=$rc" | tee -a "$OUT/session.log"
          [ $rc = 0 ] || { tail -n 20 "$OUT/${name}_r0.log"; exit 1; }
          grep -h '^{' "$OUT/${name}_r0.log" > "$OUT/$name.json" || true
          python3 tools/trace_summary.py "$OUT/$name/r0" --marker k_p2p_allreduce --top 12 \
            --json "$OUT/${name}_trace_r0.json" > "$OUT/${name}_summary.txt" 2>&1 || true
          rm -rf "$OUT/$name"
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "=== session done"
