#!/bin/bash
# rocprofv3 kernel trace of one batched series run of the native driver on the fixture of tools/series_native.py
# (run on the GPU box): tools/series_profile.sh <outdir> <series_native args...> -- <driver args...>
# e.g. tools/series_profile.sh gpurun_out/prof_sparse16 --sparse-direct -- --batch_frames 16
set -euo pipefail
out=$1; shift
gen=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do gen+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
root=$(cd "$(dirname "$0")/.." && pwd)
dir=${TMPDIR:-/tmp}/sart_series_prof
timeout -k 10 400 python -u "$root/tools/series_native.py" "${gen[@]}" --runs seq --keep --dir "$dir" \
    --out "$root/$out.gen.jsonl" > "$root/$out.gen.log" 2>&1
cd "${TMPDIR:-/tmp}"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$root/$out" -o run -- "$root/mpi_cuda_sartsolver_amd/_lib/sartsolver" \
    -m 2000 -c 1e-5 "$@" --profile "$root/$out.profile.jsonl" -o "$dir/o.h5" \
    "$dir/rtm_cam_a.h5" "$dir/rtm_cam_b.h5" "$dir/image_cam_a.h5" "$dir/image_cam_b.h5" > "$root/$out.run.log" 2>&1
rm -rf "$dir"
