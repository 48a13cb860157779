#!/usr/bin/env bash
# A/B of the N > 1 per-sweep collective on a 2-rank one-GPU rehearsal (both ranks fused on half the CUs, P2P forced):
# the P2P kernel forms the vector from the partial rows (SART_P2P_FUSED_REDUCE=1, default) against
# k_reduce_partials + the P2P all-reduce (0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
J=$OUT/ab_p2p_reduce.jsonl
for rep in 1 2; do
  for npix in 8192 32768; do
    for knob in 0 1; do
      L=$OUT/ab_p2p_${npix}_${knob}.log
      SART_P2P=1 SART_P2P_FUSED_REDUCE=$knob timeout -k 10 300 python bench.py --gpus 2 --share-gpus --steps 3 \
        --warmup 1 --npix $npix --no-selfcheck > $L 2>&1 || { echo "bench failed npix=$npix knob=$knob"; tail -20 $L; exit 1; }
      echo "{\"p2p_fused_reduce\": $knob, \"rep\": $rep, \"line\": $(tail -1 $L)}" >> $J
      python - "$J" <<'PY'
import json,sys
r=json.loads(open(sys.argv[1]).read().splitlines()[-1]); l=r["line"]
print(r["p2p_fused_reduce"], r["rep"], l["config"]["npixel_total"], l["ms_per_step"], l["iters_per_s"], l["allreduce_us_per_iter"], l["fused_sweep"], l["allreduce"][:24])
PY
    done
  done
done
