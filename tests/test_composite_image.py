"""Composite multi-camera frames (reference image.cpp:53-331; manual.pdf p.5) vs a Python oracle."""
import math

import numpy as np
import pytest

from mpi_cuda_sartsolver_amd.io import hdf5
from mpi_cuda_sartsolver_amd.io.fixtures import make_case
from mpi_cuda_sartsolver_amd.ops import native

EPS = 1e-10


def _round(x):
    return math.floor(x + 0.5)  # llround for x >= 0


def composite_oracle(timelines, intervals):
    """Pure-Python statement of the composite-frame time grid (same rules as the reference)."""
    frames, times, ctimes = [], [], []
    nc = len(timelines)
    for t0, t1, step, thr in intervals:
        sel = [[(t, i) for i, t in enumerate(tl) if t0 <= t <= t1] for tl in timelines]
        if any(not s for s in sel):
            continue
        lo = min(s[0][0] for s in sel)
        hi = max(s[-1][0] for s in sel)
        if step == 0:
            if hi - lo < EPS:
                step = 1.0
            else:
                for s in sel:
                    dmin = s[-1][0] - s[0][0]
                    for a, b in zip(s, s[1:]):
                        dmin = min(dmin, b[0] - a[0])
                    step = max(step, dmin)
                if not step > 0:
                    step = 1.0
        if thr == 0:
            thr = step
        lo -= step
        hi += step
        ng = _round((hi - lo) / step) + 1
        best = [[(1.01 * thr, 0)] * nc for _ in range(ng)]
        for c, s in enumerate(sel):
            for t, i in s:
                g0 = _round((t - lo) / step)
                for g in (g0 - 1, g0, g0 + 1):
                    if 0 <= g < ng:
                        d = t - lo - float(g) * step
                        if abs(d) + EPS < abs(best[g][c][0]):
                            best[g][c] = (d, i)
        last = 0.0
        for g in range(1, ng - 1):
            tg = lo + float(g) * step
            idx, ct, tot = [], [], 0.0
            for c in range(nc):
                d, i = best[g][c]
                if abs(d) > thr + EPS:
                    break
                idx.append(i)
                ct.append(tg + d)
                tot += abs(d)
            if len(idx) != nc:
                continue
            if not frames or idx != frames[-1]:
                frames.append(idx)
                ctimes.append(ct)
                times.append(tg)
            elif tot + EPS < last:
                times[-1] = tg
            last = tot
    return frames, times, ctimes


def _image_set(n, tmp_path, timelines, shape=(2, 2)):
    files, masks = {}, {}
    for c, tl in enumerate(timelines):
        cam = f"cam{c}"
        p = str(tmp_path / f"{cam}.h5")
        n.write_image_file(p, cam, 1.0, np.asarray(tl, float), np.zeros((len(tl),) + shape))
        files[cam] = p
        masks[cam] = np.ones(shape[0] * shape[1], np.int32)
    return files, masks


@pytest.mark.parametrize("seed", range(6))
def test_time_sync_matches_oracle(tmp_path, seed):
    n = native()
    rng = np.random.default_rng(seed)
    ncam = 1 + seed % 3
    timelines = []
    for c in range(ncam):
        dt = [0.1, 0.1, 0.05, 0.2][(seed + c) % 4]
        base = np.arange(0.0, 3.0, dt) + rng.uniform(0, 0.03)
        keep = rng.random(base.size) > 0.15
        timelines.append(np.sort(base[keep] + rng.normal(0, 0.004, keep.sum()).clip(-0.01, 0.01)))
    intervals = [[0.0, math.inf, 0.0, 0.0], [0.5, 1.7, 0.25, 0.1], [2.0, 2.9, 0.1, 0.0]][: 1 + seed % 3]
    files, masks = _image_set(n, tmp_path, timelines)
    ref_frames, ref_t, ref_ct = composite_oracle(timelines, intervals)
    if not ref_frames:
        with pytest.raises(RuntimeError, match="No composite images"):
            n.CompositeImage(files, masks, intervals, 4, 0)
        return
    ci = n.CompositeImage(files, masks, intervals, 4, 0)
    assert ci.nframe == len(ref_frames)
    assert [list(f) for f in ci.frame_indices()] == ref_frames
    for i in range(ci.nframe):
        assert ci.frame_time(i) == ref_t[i]
        assert list(ci.camera_frame_time(i)) == ref_ct[i]


def test_single_moment_and_equidistant_tie(tmp_path):
    n = native()
    files, masks = _image_set(n, tmp_path, [[1.0], [1.0]])
    ci = n.CompositeImage(files, masks, [[0.0, math.inf, 0.0, 0.0]], 4, 0)
    assert ci.nframe == 1 and ci.frame_time(0) == 1.0
    # a frame exactly between two grid points is attached to the earlier one (the '+ eps' rule)
    files, masks = _image_set(n, tmp_path, [[0.0, 1.0, 2.0], [0.5, 1.5]])
    ci = n.CompositeImage(files, masks, [[0.0, math.inf, 1.0, 0.5]], 4, 0)
    ref, _, _ = composite_oracle([[0.0, 1.0, 2.0], [0.5, 1.5]], [[0.0, math.inf, 1.0, 0.5]])
    assert [list(f) for f in ci.frame_indices()] == ref


def test_camera_without_frames_in_interval_is_skipped(tmp_path):
    n = native()
    files, masks = _image_set(n, tmp_path, [[0.0, 0.1, 0.2, 5.0, 5.1], [5.0, 5.1]])
    ci = n.CompositeImage(files, masks, [[0.0, 1.0, 0.0, 0.0], [4.9, 5.2, 0.0, 0.0]], 4, 0)
    assert all(4.9 <= ci.frame_time(i) <= 5.2 for i in range(ci.nframe)) and ci.nframe == 2


def test_unsorted_timeline_rejected(tmp_path):
    n = native()
    files, masks = _image_set(n, tmp_path, [[0.2, 0.1]])
    with pytest.raises(RuntimeError, match="not sorted by time"):
        n.CompositeImage(files, masks, [[0.0, math.inf, 0.0, 0.0]], 4, 0)


@pytest.mark.parametrize("nranks", [1, 2, 3, 5])
def test_masked_frames_and_rank_slices(tmp_path, nranks):
    from mpi_cuda_sartsolver_amd.parallel.partition import all_blocks

    case = make_case(str(tmp_path / "c"), nframes=7, saturate=0.1)
    inp = hdf5.validate_inputs(case.files)
    blocks = all_blocks(inp.npixel, nranks)
    images = [hdf5.open_composite_image(inp, [[0.0, math.inf, 0.0, 0.0]], b.size, b.offset, max_cache_size=2)
              for b in blocks]
    assert images[0].nframe == 7
    for fi in range(7):
        full = np.concatenate([im.frame(fi) for im in images])
        expect = np.concatenate([case.frames[c][fi].ravel()[case.masks[c].ravel() > 0] for c in sorted(case.masks)])
        np.testing.assert_array_equal(full, expect)
    # next_frame walks the sequence from the start
    im = hdf5.open_composite_image(inp, [[0.0, math.inf, 0.0, 0.0]], inp.npixel, 0, max_cache_size=3)
    seen = 0
    while (f := im.next_frame()) is not None:
        seen += 1
    assert seen == 7
