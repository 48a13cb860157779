#!/usr/bin/env python3
"""Split-A multi-frame projection probe: an fp32 shard on the bf16 matrix cores (k_mf_forward_b16_lds /
k_mf_backproject_b16_lds with AT = float: A split into hi + lo bf16 in registers, three products) against the
fp32 MFMA kernels (multiframe.hip), per batch width, ring depth (SART_MF_X3_DEPTH) and tile (SART_MF_X3_FWD =
"RT,KB", SART_MF_X3_VT) on a synthetic fp32 shard (default 65536 x 65536). One JSON line per measurement."""
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
    nfs = [int(v) for v in os.environ.get("PROBE_NF", "16,32,64").split(",")]
    fwd_tiles = os.environ.get("PROBE_FWD", "2,1;4,1;2,2;4,2").split(";")
    vts = os.environ.get("PROBE_VT", "1;2").split(";")
    depths = [int(v) for v in os.environ.get("PROBE_DEPTH", "2,3").split(",")]

    def emit(op, nf, med, **kw):
        print(json.dumps(dict(op=op, nf=nf, P=P, V=V, ms=round(med, 4), GBps=round(nbytes / med / 1e6, 1),
                              TFLOPs=round(2 * nf * P * V / med / 1e9, 1), **kw)), flush=True)

    for nf in nfs:
        X = torch.rand((nf, m.ld), device=dev)
        Xh = torch.empty((nf, m.ld), dtype=torch.bfloat16, device=dev)
        Xl = torch.empty_like(Xh)
        k.mf_split_x(X.data_ptr(), nf * m.ld, Xh.data_ptr(), Xl.data_ptr(), s, True)
        Fo = torch.zeros((16, m.nrows_pad, nf), device=dev)
        W = torch.rand((m.nrows_pad, nf), device=dev)
        Wh = torch.zeros((2, nf, m.nrows_pad), dtype=torch.bfloat16, device=dev)  # hi, mid (three-piece W)
        Wl = torch.zeros((nf, m.nrows_pad), dtype=torch.bfloat16, device=dev)
        k.mf_split_w(W.data_ptr(), m.nrows_pad, nf, m.nrows_pad, Wh.data_ptr(), Wl.data_ptr(), s, True)
        part = torch.zeros((64, m.ld, nf), device=dev)
        nsf = k.mf_forward_num_splits(m.ld, m.nrows_pad)
        if os.environ.get("PROBE_FP32", "1") == "1":
            med, _ = timeit(lambda: k.mf_forward(m.A.data_ptr(), m.ld, P, m.nrows_pad, X.data_ptr(), m.ld,
                                                 Fo.data_ptr(), nsf, s, nf), reps=5)
            emit("mf_forward_fp32", nf, med, nsplit=nsf)
            ns = k.mf_backproject_num_splits(m.ld, P)
            med, _ = timeit(lambda: k.mf_backproject(m.A.data_ptr(), m.ld, P, W.data_ptr(), ns, part.data_ptr(), s,
                                                     nf), reps=5)
            emit("mf_backproject_fp32", nf, med, nsplit=ns)
        for depth in depths:
            os.environ["SART_MF_X3_DEPTH"] = str(depth)
            for tile in fwd_tiles:
                os.environ["SART_MF_X3_FWD"] = tile
                med, _ = timeit(lambda: k.mf_forward_x3(m.A.data_ptr(), m.ld, P, m.nrows_pad, Xh.data_ptr(),
                                                        Xl.data_ptr(), Fo.data_ptr(), nsf, s, nf), reps=5)
                emit("mf_forward_x3", nf, med, depth=depth, tile=tile, nsplit=nsf)
            for vt in vts:
                os.environ["SART_MF_X3_VT"] = vt
                ns = k.mf_backproject_b16_num_splits(m.ld, P, True)
                assert ns <= 64
                med, _ = timeit(lambda: k.mf_backproject_x3(m.A.data_ptr(), m.ld, P, Wh.data_ptr(), Wl.data_ptr(),
                                                            m.nrows_pad, ns, part.data_ptr(), s, nf), reps=5)
                emit("mf_backproject_x3", nf, med, depth=depth, vt=vt, nsplit=ns)
        for key in ("SART_MF_X3_DEPTH", "SART_MF_X3_FWD", "SART_MF_X3_VT"):
            os.environ.pop(key, None)
        del X, Xh, Xl, Fo, W, Wh, Wl, part
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
