#!/usr/bin/env python3
"""Multi-frame MFMA projection probe: k_mf_forward / k_mf_backproject time per batch width (nf) and
register-ring depth, on a synthetic shard (default 65536 x 65536). One JSON line per measurement."""
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
    m = DenseRTM.synthetic(P, V, 0, seed=1, device=dev)
    nbytes = m.nbytes
    for nf in (16, 32, 64):
        X = torch.rand((nf, m.ld), device=dev)
        Fo = torch.zeros((16, m.nrows_pad, nf), device=dev)  # room for the split counts of either row tiling
        W = torch.rand((m.nrows_pad, nf), device=dev)
        partm = torch.zeros((16, m.ld, nf), device=dev)  # room for the split counts of either voxel tiling
        fwd_only = os.environ.get("PROBE_MF_FORWARD_ONLY") == "1"
        for depth in (1, 2, 3):
            k.mf_set_depth(depth)
            for rt in (2, 4):  # 16-row tiles per wave of the forward kernel
                k.mf_set_rows(rt)
                nsf = k.mf_forward_num_splits(m.ld, m.nrows_pad)
                assert nsf <= 16
                cases = [("mf_forward", lambda: k.mf_forward(m.A.data_ptr(), m.ld, P, m.nrows_pad, X.data_ptr(),
                                                             m.ld, Fo.data_ptr(), nsf, s, nf))]
                if not fwd_only:  # rt selects the voxel tiles of the back-projection: 1 (rt 2) or 2 (rt 4)
                    k.mf_set_vox(rt // 2)
                    nsm = k.mf_backproject_num_splits(m.ld, P)
                    assert nsm <= 16
                    cases.append(("mf_backproject", lambda: k.mf_backproject(m.A.data_ptr(), m.ld, P, W.data_ptr(),
                                                                             nsm, partm.data_ptr(), s, nf)))
                for op, fn in cases:
                    med, best = timeit(fn, reps=7)
                    print(json.dumps(dict(kind="kernel", op=op, nf=nf, depth=depth, tile=(16 * rt if op == "mf_forward" else 32 * rt), P=P, V=V,
                                          ms=round(med, 4), GBps=round(nbytes / med / 1e6, 1),
                                          TFLOPs=round(2 * nf * P * V / med / 1e9, 2))), flush=True)
        k.mf_set_depth(0)
        k.mf_set_rows(0)
        k.mf_set_vox(0)
        del X, Fo, W, partm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
