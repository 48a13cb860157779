#!/usr/bin/env python3
"""Per-tile event trace of the fused sweep (instrumented variant 6 build): where the hand-off time goes.

For every workgroup and tile the kernel stamps (s_memrealtime, 100 MHz, common to all XCDs):
  e0 compute wave 0 published its partial, e1 wave 0 obtained the weight (L steps later),
  e2 exchange stored the granule,           e3 exchange wrote the weight to LDS.
Reported (medians / p90 over tiles, microseconds):
  step       e0(t+1) - e0(t)                     pace of a workgroup
  peer_skew  max over the J peers of e2 - own e2  how late the last peer of a row group publishes
  xlat       e3 - max peer e2                     hand-off latency once the last granule exists
  wait       e1(u) - e0(u + L)                    compute wave 0 blocked on the weight
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM, fused_geometry  # noqa: E402
from mpi_cuda_sartsolver_amd.ops import hip  # noqa: E402
from mpi_cuda_sartsolver_amd.ops.state import new_state, read_state  # noqa: E402


def q(a):
    a = np.asarray(a, dtype=np.float64)
    a = a[np.isfinite(a)]
    return {"p10": round(float(np.percentile(a, 10)), 3), "med": round(float(np.median(a)), 3),
            "p90": round(float(np.percentile(a, 90)), 3), "max": round(float(a.max()), 3)} if a.size else None


def main():
    k = hip()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    ncu = int(k.device_info(0)["multiProcessorCount"])
    P, V = 65536, 65536
    m = DenseRTM.synthetic(P, V, 0, seed=1, device=dev)
    x = torch.rand(m.ld, device=dev)
    ghat = torch.rand(m.nrows_pad, device=dev)
    arow = torch.rand(m.nrows_pad, device=dev) * 1e-4
    st = new_state(dev)
    Fslot = torch.zeros(64, dtype=torch.float32, device=dev)  # [F, error word] read by decide
    xcnt = torch.zeros(16, dtype=torch.int32, device=dev)
    for T, sched in ((4, 2), (4, 4)):
        g = fused_geometry(m.ld, ncu, 6, T)
        L = 3 if sched in (0, 3) else 4
        ntile = m.nrows_pad // g.T
        nt = ntile // g.I
        part = torch.zeros(g.I * m.ld, device=dev)
        Fp = torch.zeros(2 * g.grid, dtype=torch.float64, device=dev)
        gran = torch.zeros(k.fused_granules(m.nrows_pad, g.J, g.xl), dtype=torch.int64, device=dev)
        tr = torch.zeros(g.grid * nt * 4, dtype=torch.int64, device=dev)
        k.fused_set_schedule(sched)
        k.fused_set_debug(2)
        k.fused_set_trace(tr.data_ptr(), nt)
        times = []
        for rep in range(3):
            tr.zero_()
            k.state_begin(st.data_ptr(), 1.0, 0.0, 100, s)
            k.decide(st.data_ptr(), Fslot.data_ptr(), s)
            xcnt.zero_()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            k.fused_sweep(False, g.K, g.variant, m.A.data_ptr(), m.ld, P, m.nrows_pad, x.data_ptr(), ghat.data_ptr(),
                          arow.data_ptr(), part.data_ptr(), Fp.data_ptr(), gran.data_ptr(), g.I, g.J, st.data_ptr(),
                          xcnt.data_ptr(), s)
            b.record()
            torch.cuda.synchronize()
            times.append(a.elapsed_time(b))
        k.fused_set_trace(0, 0)
        k.fused_set_debug(0)
        k.fused_set_schedule(4)
        err = read_state(st).error
        ev = tr.view(g.grid, nt, 4).cpu().numpy().astype(np.float64) / 100.0  # -> microseconds
        t0 = ev[:, 0, 0].min()
        ev -= t0
        step = np.diff(ev[:, :, 0], axis=1)
        wait = ev[:, : nt - L, 1] - ev[:, L:, 0]
        gmap = np.array(k.fused_debug_map(g.grid))
        gi_of = gmap // 1024
        out = dict(T=g.T, J=g.J, I=g.I, sched=sched, L=L, ms=float(np.median(times)), error=err, tiles=nt,
                   span_us=q(ev[:, -1, 3] - ev[:, 0, 0]), step_us=q(step), wait_us=q(wait))
        e2 = ev[:, :, 2]
        e3 = ev[:, :, 3]
        groups = [np.nonzero(gi_of == i)[0] for i in range(g.I)]
        assert all(len(grp) == g.J for grp in groups), "row groups incomplete"
        skew, xlat = [], []
        for grp in groups:
            last = e2[grp].max(axis=0)
            skew.append((last[None, :] - e2[grp]).ravel())
            xlat.append((e3[grp] - last[None, :]).ravel())
        out["peer_skew_us"] = q(np.concatenate(skew))
        out["xlat_us"] = q(np.concatenate(xlat))
        out["e0_to_e2_us"] = q((e2 - ev[:, :, 0]).ravel())
        out["e3_to_e1_us"] = q((ev[:, :, 1] - e3).ravel())  # weight ready -> used (slack left, >= 0)
        e0 = ev[:, :, 0]
        out["peer_e0_spread_us"] = q(np.concatenate([(e0[grp].max(0) - e0[grp].min(0)) for grp in groups]))
        print(json.dumps(out), flush=True)
        np.save(f"gpurun_out/fused_trace_T{g.T}_s{sched}.npy", ev.astype(np.float32))
        del part, gran, tr


if __name__ == "__main__":
    main()
