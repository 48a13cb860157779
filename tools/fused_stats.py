#!/usr/bin/env python3
"""Diagnostic: where the fused sweep (variant 4) spends its time (s_memtime stamps, dbg flag 2)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM, fused_geometry  # noqa: E402
from mpi_cuda_sartsolver_amd.ops import hip  # noqa: E402
from mpi_cuda_sartsolver_amd.ops.state import new_state, read_state  # noqa: E402


VARIANT = int(os.environ.get('SART_FUSED_VARIANT', '6'))


def main():
    k = hip()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    ncu = int(k.device_info(0)["multiProcessorCount"])
    for arg in sys.argv[1:] or ["65536x65536"]:
        P, V = (int(v) for v in arg.split("x"))
        m = DenseRTM.synthetic(P, V, 0, seed=1, device=dev)
        g = fused_geometry(m.ld, ncu, VARIANT)
        x = torch.rand(m.ld, device=dev)
        ghat = torch.rand(m.nrows_pad, device=dev)
        arow = torch.rand(m.nrows_pad, device=dev) * 1e-4
        part = torch.zeros(g.I * m.ld, device=dev)
        Fp = torch.zeros(2 * g.grid, dtype=torch.float64, device=dev)
        gran = torch.zeros(k.fused_granules(m.nrows_pad, g.J, g.xl), dtype=torch.int64, device=dev)
        st = new_state(dev)
        Fslot = torch.zeros(64, dtype=torch.float32, device=dev)  # [F, error word] read by decide
        xcnt = torch.zeros(16, dtype=torch.int32, device=dev)
        for flags in (2, 3):
            k.fused_set_debug(flags)
            times = []
            for rep in range(4):
                k.state_begin(st.data_ptr(), 1.0, 0.0, 100, s)
                k.decide(st.data_ptr(), Fslot.data_ptr(), s)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                xcnt.zero_()
                k.fused_sweep(False, g.K, g.variant, m.A.data_ptr(), m.ld, P, m.nrows_pad, x.data_ptr(), ghat.data_ptr(),
                              arow.data_ptr(), part.data_ptr(), Fp.data_ptr(), gran.data_ptr(), g.I, g.J,
                              st.data_ptr(), xcnt.data_ptr(), s)
                b.record()
                torch.cuda.synchronize()
                times.append(a.elapsed_time(b))
            stats = np.array(k.fused_debug_stats(g.grid), dtype=np.float64).reshape(g.grid, 8)
            loop = stats[:, 4]
            out = dict(P=P, V=V, flags=flags, ms=float(np.median(times)), err=read_state(st).error,
                       loop_cycles_med=float(np.median(loop)),
                       stall_frac_wave=[float(np.median(stats[:, w] / loop)) for w in range(4)],
                       stall_frac_max=float(np.max(stats[:, 0] / loop)),
                       stalled_steps_med=float(np.median(stats[:, 5])),
                       xwait_frac_med=float(np.median(stats[:, 6] / loop)), repolls_med=float(np.median(stats[:, 7])),
                       repolls_max=float(np.max(stats[:, 7])), steps=int(m.nrows_pad // 4 // g.I))
            print(json.dumps(out), flush=True)
        k.fused_set_debug(0)
        del m, gran, part
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
