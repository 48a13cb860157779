#!/usr/bin/env python3
"""Per-kernel timing probe on one GPU (HIP events): achievable HBM roof vs our projection kernels.

Prints one JSON line per measurement: kernel, shape, ms, effective GB/s.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM, fused_geometry  # noqa: E402
from mpi_cuda_sartsolver_amd.ops import hip  # noqa: E402
from mpi_cuda_sartsolver_amd.ops.state import new_state  # noqa: E402


def timeit(fn, reps=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in evs)
    return ts[len(ts) // 2], ts[0]


def emit(**kw):
    print(json.dumps(kw), flush=True)


def main():
    k = hip()
    dev = torch.device("cuda", 0)
    info = k.device_info(0)
    emit(kind="device", **{kk: (v if not isinstance(v, bytes) else v.decode()) for kk, v in info.items()})
    s = torch.cuda.current_stream().cuda_stream
    shapes = [(65536, 65536), (16384, 65536), (65536, 16384), (8192, 262144)]
    if len(sys.argv) > 1:
        shapes = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]]

    # HBM roof: device-to-device copy of 4 GiB (read + write) and a torch sum (read only)
    buf = torch.empty(1 << 30, dtype=torch.float32, device=dev)
    buf2 = torch.empty_like(buf)
    med, best = timeit(lambda: buf2.copy_(buf), reps=5)
    emit(kind="roof", op="copy_4GiB", ms=med, GBps=2 * buf.numel() * 4 / med / 1e6, best_GBps=2 * buf.numel() * 4 / best / 1e6)
    med, best = timeit(lambda: buf.sum(), reps=5)
    emit(kind="roof", op="torch.sum_4GiB", ms=med, GBps=buf.numel() * 4 / med / 1e6, best_GBps=buf.numel() * 4 / best / 1e6)
    del buf, buf2
    torch.cuda.empty_cache()

    for (P, V) in shapes:
        t0 = time.time()
        m = DenseRTM.synthetic(P, V, 0, seed=1, device=dev)
        torch.cuda.synchronize()
        emit(kind="synth", P=P, V=V, ld=m.ld, s=time.time() - t0, GB=m.nbytes / 1e9)
        nbytes = m.nbytes
        x = torch.rand(m.ld, device=dev)
        x[V:] = 0
        ghat = torch.rand(m.nrows_pad, device=dev)
        arow = torch.rand(m.nrows_pad, device=dev) * 1e-4
        w = torch.zeros(m.nrows_pad, device=dev)
        nb = k.forward_num_blocks(m.nrows_pad)
        Fp = torch.zeros(max(nb, 8192), dtype=torch.float64, device=dev)
        st = new_state(dev)
        Fslot = torch.zeros(64, dtype=torch.float32, device=dev)  # [F, error word] read by decide
        k.state_begin(st.data_ptr(), 1.0, 0.0, 100, s)

        def fwd():
            k.forward(1, m.A.data_ptr(), m.ld, P, m.nrows_pad, x.data_ptr(), ghat.data_ptr(), arow.data_ptr(), 0,
                      w.data_ptr(), Fp.data_ptr(), 0, s)

        med, best = timeit(fwd)
        emit(kind="kernel", op="forward_lin", P=P, V=V, ms=med, GBps=nbytes / med / 1e6, best_GBps=nbytes / best / 1e6)

        ns = k.backproject_num_splits(m.ld, P)
        part = torch.zeros(max(ns, 64) * m.ld, device=dev)

        def bwd():
            k.backproject(m.A.data_ptr(), m.ld, P, ghat.data_ptr(), ns, part.data_ptr(), 0, s)

        med, best = timeit(bwd)
        emit(kind="kernel", op="backproject", P=P, V=V, nsplit=ns, ms=med, GBps=nbytes / med / 1e6,
             best_GBps=nbytes / best / 1e6)

        cfgs = [(6, 4, 4), (6, 2, 4), (6, 1, 4), (6, 4, 2), (6, 4, 0), (3, None, 0)]
        if os.environ.get("PROBE_CFGS"):  # e.g. "6:4:4,6:1:4,3:0:0"
            cfgs = [tuple((int(v) or None) if i == 1 else int(v) for i, v in enumerate(c.split(":")))
                    for c in os.environ["PROBE_CFGS"].split(",")]
        for variant, T, sched in cfgs:
            g = fused_geometry(m.ld, int(info["multiProcessorCount"]), variant, T)
            if g is None or g.variant != variant or (T is not None and g.T != T):
                continue
            gran = torch.zeros(k.fused_granules(m.nrows_pad, g.J, g.xl), dtype=torch.int64, device=dev)
            xcnt = torch.zeros(16, dtype=torch.int32, device=dev)
            if part.numel() < g.I * m.ld:
                part = torch.zeros(g.I * m.ld, device=dev)

            def fused():
                k.fused_set_schedule(sched if sched is not None else 4)
                xcnt.zero_()
                k.state_begin(st.data_ptr(), 1.0, 0.0, 100, s)
                k.decide(st.data_ptr(), Fslot.data_ptr(), s)  # sweep 0 -> epoch+1, not done
                k.fused_sweep(False, g.K, g.variant, m.A.data_ptr(), m.ld, P, m.nrows_pad, x.data_ptr(),
                              ghat.data_ptr(), arow.data_ptr(), part.data_ptr(), Fp.data_ptr(), gran.data_ptr(),
                              g.I, g.J, st.data_ptr(), xcnt.data_ptr(), s)

            med, best = timeit(fused)
            from mpi_cuda_sartsolver_amd.ops.state import read_state

            err = read_state(st).error
            tag = f"fused_sweep_v{variant}" + (f"_T{g.T}" if variant in (4, 6) else "") + (f"_s{sched}" if sched else "")
            emit(kind="kernel", op=tag, P=P, V=V, K=g.K, J=g.J, I=g.I, T=g.T, ms=med,
                 GBps=nbytes / med / 1e6, best_GBps=nbytes / best / 1e6, error=err)
            k.fused_set_debug(1)
            med, best = timeit(fused)
            k.fused_set_debug(0)
            emit(kind="kernel", op=f"{tag}_noexchange", P=P, V=V, ms=med, GBps=nbytes / med / 1e6)
            k.fused_set_schedule(4)
            del gran

        if os.environ.get("PROBE_FUSED_ONLY"):
            del m, part
            torch.cuda.empty_cache()
            continue
        # multi-frame MFMA projections (16 frames)
        X = torch.rand((16, m.ld), device=dev)
        nsf = k.mf_forward_num_splits(m.ld, m.nrows_pad)
        Fo = torch.zeros((nsf, m.nrows_pad, 16), device=dev)
        med, best = timeit(lambda: k.mf_forward(m.A.data_ptr(), m.ld, P, m.nrows_pad, X.data_ptr(), m.ld,
                                                Fo.data_ptr(), nsf, s))
        emit(kind="kernel", op="mf_forward16", P=P, V=V, ms=med, GBps=nbytes / med / 1e6,
             TFLOPs=2 * 16 * P * V / med / 1e9)
        W = torch.rand((m.nrows_pad, 16), device=dev)
        nsm = k.mf_backproject_num_splits(m.ld, P)
        partm = torch.zeros((nsm, m.ld, 16), device=dev)
        med, best = timeit(lambda: k.mf_backproject(m.A.data_ptr(), m.ld, P, W.data_ptr(), nsm, partm.data_ptr(), s))
        emit(kind="kernel", op="mf_backproject16", P=P, V=V, ms=med, GBps=nbytes / med / 1e6,
             TFLOPs=2 * 16 * P * V / med / 1e9)
        del m, part, partm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
