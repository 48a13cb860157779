#!/usr/bin/env python3
"""Infinity-cache (MALL) reuse probe for the multi-frame engine: can the back-projection re-read a row block of
A from the 256 MB memory-side cache when it runs right after the forward of the same block?

Prints JSON lines: the read rate of a tensor re-read while it is cache resident (torch.sum, 32 MB .. 1 GB), the
full two-pass 16-frame sweep (forward + back-projection over all rows), and row-blocked sweeps (forward then
back-projection per block of R rows) at several R. Timing only: the outputs are scratch.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM  # noqa: E402
from mpi_cuda_sartsolver_amd.ops import hip  # noqa: E402
from probe import emit, timeit  # noqa: E402


def main():
    k = hip()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    for mb in (32, 64, 128, 192, 256, 512, 1024, 4096):
        t = torch.ones(mb * (1 << 20) // 4, device=dev)
        med, best = timeit(lambda: t.sum(), reps=20, warm=3)
        emit(kind="resident_read", MB=mb, ms=med, GBps=t.numel() * 4 / med / 1e6)
        del t
    torch.cuda.empty_cache()

    P, V = 65536, 65536
    nf = 16
    m = DenseRTM.synthetic(P, V, 0, seed=1, device=dev)
    ld, Pp = m.ld, m.nrows_pad
    gb = m.nbytes / 1e9
    X = torch.rand((nf, ld), device=dev)
    W = torch.rand((Pp, nf), device=dev)
    Fo = torch.zeros((64, Pp, nf), device=dev)
    part = torch.zeros((64, ld, nf), device=dev)
    A0 = m.A.data_ptr()
    for rt in (1, 2, 4):
        k.mf_set_rows(rt)
        nsf = k.mf_forward_num_splits(ld, Pp)
        nsb = k.mf_backproject_num_splits(ld, P)
        assert nsf <= 64 and nsb <= 64

        def full():
            k.mf_forward(A0, ld, P, Pp, X.data_ptr(), ld, Fo.data_ptr(), nsf, s, nf)
            k.mf_backproject(A0, ld, P, W.data_ptr(), nsb, part.data_ptr(), s, nf)

        med, best = timeit(full, reps=5)
        emit(kind="full_two_pass", rt=rt, nsf=nsf, nsb=nsb, ms=med, TBps_2reads=2 * gb / med)
        for R in (256, 512, 1024, 2048):
            nsf_b = k.mf_forward_num_splits(ld, R)
            nsb_b = k.mf_backproject_num_splits(ld, R)
            if nsf_b > 64 or nsb_b > 64:
                continue

            def blocked(bwd=True):
                for r0 in range(0, P, R):
                    a = A0 + r0 * ld * 4
                    k.mf_forward(a, ld, R, R, X.data_ptr(), ld, Fo.data_ptr(), nsf_b, s, nf)
                    if bwd:
                        k.mf_backproject(a, ld, R, W.data_ptr() + r0 * nf * 4, nsb_b, part.data_ptr(), s, nf)

            med, best = timeit(blocked, reps=3, warm=1)
            medf, _ = timeit(lambda: blocked(False), reps=3, warm=1)
            emit(kind="row_blocked", rt=rt, R=R, block_MB=R * ld * 4 / 2**20, nsf=nsf_b, nsb=nsb_b, ms=med,
                 fwd_only_ms=medf, bwd_ms=med - medf, TBps_2reads=2 * gb / med, fwd_TBps=gb / medf)


if __name__ == "__main__":
    main()
