#!/usr/bin/env python3
"""Time-series throughput of the native driver (the reference's product: a warm-started frame loop timed by
"Processed in", reference main.cpp:127-140) at 64k x 64k on HDF5 files.

Writes two cameras' dense RTMs (32768 pixels x 65536 voxels each, 17.2 GB together) and an image series of --frames
frames per camera, computed on the GPU from the same matrix:

* default: the ray-traced camera model with wall reflections (utils/raytrace.py, 32 x 32 x 64 voxels, two 128 x 256
  cameras) and its drifting ring phantom (t advancing --tstep per frame), written with the dense RTM writer;
* --random: the uniform random dense RTM of the load bench (native streaming writer) with x_t = b (1 + amp sin(2 pi
  t / period + phase_v)) -- SART converges on it within 2-3 sweeps whatever the start, so it times overheads only.

Then runs ``sartsolver --profile`` over the series (default stopping rule, fused sweep) and a calibration run of one frame
with a fixed iteration count (the per-sweep time t_sweep). Reports frames/s, the "Processed in" distribution and
the per-frame overhead beyond sweeps x t_sweep, with the driver's own breakdown (setup: normalisation + H2D of g and
x0; iterate; finish: D2H of x + de-normalisation; writer; frame reads the prefetch did not hide), one JSON line per
run. The fixture files are written in this process, so their reads are page-cache reads.
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _all_recs(d, tag):
    p = os.path.join(d, f"prof_{tag}.jsonl")
    return [json.loads(x) for x in open(p)] if os.path.exists(p) else []


def pct(a, q):
    return float(np.percentile(np.asarray(a, dtype=float), q)) if len(a) else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp") + "/sart_series")
    ap.add_argument("--h", type=int, default=128)
    ap.add_argument("--w", type=int, default=256)
    ap.add_argument("--nvox", type=int, default=65536)
    ap.add_argument("--frames", type=int, default=240)
    ap.add_argument("--amp", type=float, default=0.05)
    ap.add_argument("--period", type=float, default=200.0)
    ap.add_argument("--random", action="store_true", help="uniform random RTM instead of the ray-traced one")
    ap.add_argument("--sparse-direct", action="store_true",
                    help="the ray-traced model's direct (no-reflection) part, written as sparse COO files: the driver "
                         "keeps it sparse on the GPU (--rtm_format auto)")
    ap.add_argument("--tstep", type=float, default=0.1, help="phantom time step per frame (ray-traced)")
    ap.add_argument("--runs", default="seq", help="comma list: seq (frame by frame), batch<N> (--batch_frames N)")
    ap.add_argument("--extra", default="", help="extra driver arguments for every run")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "series_native.jsonl"))
    ap.add_argument("--batch-sweep-ms", type=float, default=0.0,
                    help="time of one batched sweep (tools/probe_mf.py) for the sweeps x t_sweep / loop figure")
    ap.add_argument("--keep", action="store_true")
    a = ap.parse_args()
    import torch

    from mpi_cuda_sartsolver_amd.io.hdf5 import load_rtm_shard, validate_inputs
    from mpi_cuda_sartsolver_amd.ops import native

    n = native()
    binary = os.path.join(ROOT, "mpi_cuda_sartsolver_amd", "_lib", "sartsolver")
    os.makedirs(a.dir, exist_ok=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    outf = open(a.out, "a")

    def emit(rec):
        line = json.dumps(rec)
        print(line, flush=True)
        outf.write(line + "\n")
        outf.flush()

    t0 = time.perf_counter()
    cams = ["cam_a", "cam_b"]
    rtm = [os.path.join(a.dir, f"rtm_{c}.h5") for c in cams]
    dev = torch.device("cuda", 0)
    times = 0.01 * np.arange(a.frames)
    P1 = a.h * a.w
    if a.random:
        for c, path in zip(cams, rtm):
            n.write_synthetic_rtm_file(path, c, 656.3, a.h, a.w, a.nvox, seed=7 + len(c) + ord(c[-1]), nnz_per_row=0,
                                       drop_cache=False)
        t_rtm = time.perf_counter() - t0
        # frames: G = A X^T on the GPU, from the matrix as the driver will read it
        tmp_img = [os.path.join(a.dir, f"img0_{c}.h5") for c in cams]
        for c, path in zip(cams, tmp_img):  # a one-frame placeholder so the reader can validate the set
            n.write_image_file(path, c, 657.3, np.array([0.0]), np.ones((1, a.h, a.w)))
        inp = validate_inputs(rtm + tmp_img)
        shard = load_rtm_shard(inp, 0, inp.npixel, dev)
        rng = np.random.default_rng(3)
        b = 0.5 + rng.random(a.nvox)
        ph = 2 * np.pi * rng.random(a.nvox)
        X = np.stack([b * (1 + a.amp * np.sin(2 * np.pi * t / a.period + ph)) for t in range(a.frames)])
        Ad = shard.A[: inp.npixel, : a.nvox]
        model = "uniform random dense (native writer)"
        phantom_desc = f"b (1 + {a.amp} sin(2 pi t / {a.period} + phase))"
    elif a.sparse_direct:
        from mpi_cuda_sartsolver_amd.models.rtm import SparseRTM
        from mpi_cuda_sartsolver_amd.models.sart import SARTSolver
        from mpi_cuda_sartsolver_amd.utils.raytrace import Camera, default_cameras, phantom, raytraced_direct_coo

        grids = {4096: (16, 16, 16), 32768: (32, 32, 32), 65536: (32, 32, 64)}
        grid = grids[a.nvox]
        cobj = [Camera(c, bc.position, bc.look_at, (a.h, a.w), bc.field_of_view, bc.up)
                for c, bc in zip(cams, default_cameras(n=2))]
        r, c, v, info = raytraced_direct_coo(grid=grid, cameras=cobj)
        flat = np.arange(a.nvox)
        nx, ny, nz = grid
        vi, vj, vk = flat // (ny * nz), (flat // nz) % ny, flat % nz
        for cam, path in zip(cams, rtm):
            r0, r1 = info[cam]
            sel = (r >= r0) & (r < r1)
            n.write_rtm_file(path=path, camera_name=cam, wavelength=656.3, npixel=r1 - r0, nvoxel=a.nvox,
                             frame_mask=np.ones((a.h, a.w), np.uint8), vi=vi.astype(np.uint64), vj=vj.astype(np.uint64),
                             vk=vk.astype(np.uint64), vvalue=np.arange(a.nvox, dtype=np.int32), nx=nx, ny=ny, nz=nz,
                             rtm_name="with_reflections", coordinate_system="", bounds=[],
                             pixel_index=(r[sel] - r0).astype(np.uint64), voxel_index=c[sel].astype(np.uint64),
                             value=v[sel])
        t_rtm = time.perf_counter() - t0
        X = np.stack([phantom(grid, t=a.tstep * k) for k in range(a.frames)])
        sp = SparseRTM.from_entries(2 * P1, a.nvox, r, c, v, device=dev)
        fwd = SARTSolver(sp)
        G = np.stack([fwd.forward_project(X[k]) for k in range(a.frames)])
        del fwd, sp
        model = "ray-traced direct part (no reflections), sparse COO files"
        phantom_desc = f"utils.raytrace.phantom(t = {a.tstep} k)"
        Xd = None
    else:
        from mpi_cuda_sartsolver_amd.utils.raytrace import Camera, default_cameras, phantom, raytraced_rtm

        grids = {4096: (16, 16, 16), 32768: (32, 32, 32), 65536: (32, 32, 64)}
        if a.nvox not in grids:
            raise SystemExit(f"ray-traced series: --nvox one of {sorted(grids)}")
        grid = grids[a.nvox]
        base_cams = default_cameras(n=2)
        cobj = [Camera(c, bc.position, bc.look_at, (a.h, a.w), bc.field_of_view, bc.up) for c, bc in zip(cams, base_cams)]
        A, info = raytraced_rtm(grid=grid, cameras=cobj, keep_direct=False)
        flat = np.arange(a.nvox)
        nx, ny, nz = grid
        vi, vj, vk = flat // (ny * nz), (flat // nz) % ny, flat % nz
        for c, path in zip(cams, rtm):
            r0, r1 = info["rows"][c]
            n.write_rtm_file(path=path, camera_name=c, wavelength=656.3, npixel=r1 - r0, nvoxel=a.nvox,
                             frame_mask=np.ones((a.h, a.w), np.uint8), vi=vi.astype(np.uint64), vj=vj.astype(np.uint64),
                             vk=vk.astype(np.uint64), vvalue=np.arange(a.nvox, dtype=np.int32), nx=nx, ny=ny, nz=nz,
                             rtm_name="with_reflections", coordinate_system="", bounds=[],
                             dense=np.ascontiguousarray(A[r0:r1]))
        t_rtm = time.perf_counter() - t0
        X = np.stack([phantom(grid, t=a.tstep * k) for k in range(a.frames)])
        Ad = torch.from_numpy(A).to(dev)
        del A
        model = "ray-traced with reflections (utils/raytrace.py)"
        phantom_desc = f"utils.raytrace.phantom(t = {a.tstep} k)"
    if not a.sparse_direct:
        Xd = torch.from_numpy(X.T.astype(np.float32)).to(dev)
        G = (Ad @ Xd).double().cpu().numpy().T  # [frames, pixels]
        del Ad, Xd
    torch.cuda.empty_cache()
    img = [os.path.join(a.dir, f"image_{c}.h5") for c in cams]
    for k, (c, path) in enumerate(zip(cams, img)):
        n.write_image_file(path, c, 657.3, times, G[:, k * P1:(k + 1) * P1].reshape(a.frames, a.h, a.w))
    fixture_s = time.perf_counter() - t0
    files = rtm + img
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    base = {"npixel": 2 * P1, "nvoxel": a.nvox, "frames": a.frames, "cameras": 2,
            "rtm_GB": (r.size * 16 / 1e9) if a.sparse_direct else 2 * P1 * a.nvox * 4 / 1e9,
            "rtm": model, "phantom": phantom_desc, "fixture_s": round(fixture_s, 1),
            "rtm_write_s": round(t_rtm, 1), "reads": "page cache (files written by this process)"}
    extra = a.extra.split() if a.extra else []

    def drive(tag, argv, env_over=None):
        prof = os.path.join(a.dir, f"prof_{tag}.jsonl")
        out = os.path.join(a.dir, f"sol_{tag}.h5")
        t = time.perf_counter()
        r = subprocess.run([binary, *argv, *extra, "--profile", prof, "-o", out, *files], env=dict(env, **(env_over or {})),
                           capture_output=True, text=True, timeout=1500)
        wall = time.perf_counter() - t
        if r.returncode != 0:
            raise RuntimeError(f"{tag}: rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}")
        recs = [json.loads(x) for x in open(prof)]
        recs = [x for x in recs if not x.get("series")] + [x for x in recs if x.get("series")]
        m = re.search(r"Frames processed: (\d+) in ([0-9.eE+-]+) s", r.stdout)
        return recs[0], [x for x in recs[1:] if "frame" in x], wall, (float(m.group(2)) if m else None), r.stdout

    # calibration: frame 0 cold, 200 iterations with a tolerance that never fires on this matrix -> the time per
    # sweep of the solve loop (iterate_ms over the sweeps; the few no-op sweeps queued past the last one are
    # counted at zero, which errs towards a larger per-sweep time, i.e. a smaller overhead, by < 1 %)
    _, cal, _, _, _ = drive("cal", ["-m", "200", "-c", "1e-30", "-t", "0:0.005"])
    t_sweep = cal[0]["iterate_ms"] / cal[0]["sweeps"]
    sols = {}
    t_sweep_of = []
    if a.batch_sweep_ms:  # the batched sweep time (per batch width) for the loop-share figure
        t_sweep_of.append(a.batch_sweep_ms)
    emit(dict(base, run="calibration", sweeps=cal[0]["sweeps"], queued=cal[0]["queued_sweeps"],
              iterate_ms=cal[0]["iterate_ms"], t_sweep_ms=round(t_sweep, 4),
              valid=cal[0]["sweeps"] >= 100))
    for run in a.runs.split(","):
        # a run: seq | batch<N>, optionally @VAR=value+VAR=value (environment of that run: A/B knobs)
        spec, _, envs = run.partition("@")
        env_over = dict(kv.split("=", 1) for kv in envs.split("+")) if envs else {}
        argv = ["-m", "2000", "-c", "1e-5"]
        if spec.startswith("batch"):
            argv += ["--batch_frames", spec[5:]]
        run = run.replace("@", "_").replace("+", "_").replace("=", "")
        load, fr, wall, loop_s, _ = drive(run, argv, env_over)
        ms = [x["ms"] for x in fr]
        rec = dict(base, run=run, process_wall_s=round(wall, 2), load_s=round(load.get("load_s", 0), 2),
                   load_GBps=round(load.get("load_GBps", 0), 2), load_rss_growth_MB=load.get("rss_growth_MB_max"),
                   load_staging_MB=load.get("rank0", {}).get("staging_MB"),
                   loop_s=loop_s, frames_per_s=round(len(fr) / loop_s, 2) if loop_s else None,
                   processed_ms={"mean": round(float(np.mean(ms)), 3), "p50": round(pct(ms, 50), 3),
                                 "p90": round(pct(ms, 90), 3), "p99": round(pct(ms, 99), 3),
                                 "max": round(max(ms), 3), "min": round(min(ms), 3)},
                   iterations={"mean": round(float(np.mean([x["iterations"] for x in fr])), 2),
                               "p50": pct([x["iterations"] for x in fr], 50),
                               "max": max(x["iterations"] for x in fr),
                               "first": fr[0]["iterations"]},
                   converged=sum(x["status"] == 0 for x in fr))
        series = [x for x in [load, *fr] if x.get("series")] + [x for x in _all_recs(a.dir, run) if x.get("series")]
        if series:  # batched: the device-refill counters (sweeps, slot utilisation, chain sources)
            rec["series"] = series[-1]
            rec["sweeps_x_t_sweep_over_loop"] = round(series[-1]["sweeps"] * t_sweep_of[0] / 1e3 / loop_s, 3) \
                if t_sweep_of and loop_s else None
        sols[run] = n.read_dataset_f64(os.path.join(a.dir, f"sol_{run}.h5"), "solution/value")
        rec["env"] = env_over
        if X is not None and sols[run].shape == X.shape:  # every frame against the phantom it was computed from
            d = np.linalg.norm(sols[run] - X, axis=1) / np.linalg.norm(X, axis=1)
            rec["rel_err_vs_truth"] = {"p50": pct(d, 50), "p90": pct(d, 90), "max": float(d.max()),
                                       "mean": float(d.mean())}
        if run != "seq" and "seq" in sols:  # every frame against the sequential chain's solution
            ref = sols["seq"]
            d = np.linalg.norm(sols[run] - ref, axis=1) / np.maximum(np.linalg.norm(ref, axis=1), 1e-300)
            rec["rel_diff_vs_seq"] = {"p50": pct(d, 50), "p90": pct(d, 90), "p99": pct(d, 99), "max": float(d.max())}
        if "sweeps" in fr[0]:  # frame by frame: overhead beyond the sweeps actually needed
            over = [x["ms"] - x["sweeps"] * t_sweep for x in fr[1:]]  # warm-started frames
            keys = ("setup_ms", "iterate_ms", "finish_ms", "writer_ms", "wait_frame_ms")
            rec.update(
                t_sweep_ms=round(t_sweep, 4),
                overhead_ms={"mean": round(float(np.mean(over)), 3), "p50": round(pct(over, 50), 3),
                             "p90": round(pct(over, 90), 3), "max": round(max(over), 3)},
                breakdown_mean_ms={k: round(float(np.mean([x[k] for x in fr[1:]])), 4) for k in keys},
                breakdown_max_ms={k: round(float(np.max([x[k] for x in fr[1:]])), 4) for k in keys},
                queued_minus_sweeps_mean=round(float(np.mean([x["queued_sweeps"] - x["sweeps"] for x in fr[1:]])), 2),
                iterate_minus_sweeps_ms_mean=round(float(np.mean([x["iterate_ms"] - x["sweeps"] * t_sweep
                                                                   for x in fr[1:]])), 3))
        emit(rec)
    if not a.keep:
        shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
