#!/usr/bin/env bash
# A/B of the one-rank SART iteration tail: reduce + decide + update in one kernel (default) against three
# launches (SART_TAIL_FUSED=0), at the headline shard and at 1/8 and 1/4 of it; then kernel statistics.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
J=$OUT/ab_tail.jsonl
for rep in 1 2; do
  for npix in 65536 8192 16384; do
    for knob in 0 1; do
      SART_TAIL_FUSED=$knob timeout -k 10 240 python bench.py --steps 5 --warmup 1 --npix $npix --no-selfcheck \
        > $OUT/ab_tail_${npix}_${knob}.log 2>&1 || { echo "bench failed npix=$npix knob=$knob"; tail -20 $OUT/ab_tail_${npix}_${knob}.log; exit 1; }
      echo "{\"tail_fused\": $knob, \"rep\": $rep, \"line\": $(tail -1 $OUT/ab_tail_${npix}_${knob}.log)}" >> $J
      python - "$J" <<'PY'
import json,sys
r=json.loads(open(sys.argv[1]).read().splitlines()[-1]); l=r["line"]
print(r["tail_fused"], r["rep"], l["config"]["npixel_total"], l["ms_per_step"], l["iters_per_s"], l["effective_hbm_TBps_per_gpu"])
PY
    done
  done
done
