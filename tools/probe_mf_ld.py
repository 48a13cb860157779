#!/usr/bin/env python3
"""Row-stride probe of the bf16 multi-frame projections: k_mf_forward_b16 / k_mf_backproject_b16 at 64 frames on a
synthetic bf16 shard whose row pitch ld is the voxel count plus PROBE_LD_EXTRA columns (default 0, 64, 128, 256,
1024). The MFMA fragments read 64 or 128 bytes of many rows per instruction, so a power-of-two pitch may put every
row of a step on the same HBM channel. One JSON line per (ld, kernel)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM  # noqa: E402
from mpi_cuda_sartsolver_amd.ops import hip  # noqa: E402
from probe import timeit  # noqa: E402


def main():
    k = hip()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    P, V = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "65536x65536").split("x"))
    nf = int(os.environ.get("PROBE_NF", "64"))
    for extra in [int(v) for v in os.environ.get("PROBE_LD_EXTRA", "0,64,128,256,1024").split(",")]:
        m = DenseRTM.synthetic(P, V, 0, seed=1, device=dev, storage="bf16", ld=V + extra)
        nbytes = P * V * 2
        Xh = torch.rand((nf, m.ld), device=dev).bfloat16()
        Xl = (torch.rand((nf, m.ld), device=dev) * 1e-3).bfloat16()
        nsf = k.mf_forward_num_splits(m.ld, m.nrows_pad)
        Fo = torch.zeros((nsf, m.nrows_pad, nf), device=dev)
        Wh = torch.rand((nf, m.nrows_pad), device=dev).bfloat16()
        Wl = (torch.rand((nf, m.nrows_pad), device=dev) * 1e-3).bfloat16()
        ns = k.mf_backproject_b16_num_splits(m.ld, P)
        part = torch.zeros((ns, m.ld, nf), device=dev)
        med, _ = timeit(lambda: k.mf_forward_b16(m.A.data_ptr(), m.ld, P, m.nrows_pad, Xh.data_ptr(), Xl.data_ptr(),
                                                 Fo.data_ptr(), nsf, s, nf), reps=5)
        print(json.dumps(dict(op="mf_forward_b16", nf=nf, P=P, V=V, ld=m.ld, nsplit=nsf, ms=round(med, 4),
                              GBps=round(nbytes / med / 1e6, 1))), flush=True)
        med, _ = timeit(lambda: k.mf_backproject_b16(m.A.data_ptr(), m.ld, P, Wh.data_ptr(), Wl.data_ptr(),
                                                     m.nrows_pad, ns, part.data_ptr(), s, nf), reps=5)
        print(json.dumps(dict(op="mf_backproject_b16", nf=nf, P=P, V=V, ld=m.ld, nsplit=ns, ms=round(med, 4),
                              GBps=round(nbytes / med / 1e6, 1))), flush=True)
        del m, Xh, Xl, Fo, Wh, Wl, part
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
