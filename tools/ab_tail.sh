#!/usr/bin/env bash
# A/B of the one-rank SART iteration tail at the headline shard and at 1/8 and 1/4 of it. Arguments: env settings
# to compare (default: SART_TAIL_FUSED=0, the three-launch tail, against SART_TAIL_FUSED=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
J=$OUT/ab_tail.jsonl
[ $# -gt 0 ] || set -- SART_TAIL_FUSED=0 SART_TAIL_FUSED=1
for rep in 1 2; do
  for npix in 65536 8192 16384; do
    for knob in "$@"; do
      L=$OUT/ab_tail_${npix}_${knob//=/_}.log
      env $knob timeout -k 10 240 python bench.py --steps 5 --warmup 1 --npix $npix --no-selfcheck > $L 2>&1 \
        || { echo "bench failed npix=$npix $knob"; tail -20 $L; exit 1; }
      echo "{\"env\": \"$knob\", \"rep\": $rep, \"line\": $(tail -1 $L)}" >> $J
      python - "$J" <<'PY'
import json,sys
r=json.loads(open(sys.argv[1]).read().splitlines()[-1]); l=r["line"]
print(r["env"], r["rep"], l["config"]["npixel_total"], l["ms_per_step"], l["iters_per_s"], l["effective_hbm_TBps_per_gpu"])
PY
    done
  done
done
