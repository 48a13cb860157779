#!/usr/bin/env python3
"""Ablations of the split-A 64-frame back-projection (k_mf_backproject_b16_lds<4, 2, 1, float, ABL>, the bf16
three-piece form): time per call with the MFMAs (1), the in-register split of A (2) and / or the W staging + barrier
(4) removed (SART_MF_ABL = OR of the bits), on a synthetic fp32 shard (default 65536 x 65536); the bit whose removal
moves the time names the pipe that bounds a step. Then back-projection variants (PROBE_BWD, "lds" = the bf16 form,
"h16[+ew|w1]" = the f16-pair kernel, "_vt2" two voxel tiles per wave) against the first, and the split-A forward's
ablations. One JSON line per variant."""
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
    nf = 64
    m = DenseRTM.synthetic(P, V, 0, seed=1, device=dev)
    W = torch.rand((m.nrows_pad, nf), device=dev)
    Wh = torch.zeros((2, nf, m.nrows_pad), dtype=torch.bfloat16, device=dev)
    Wl = torch.zeros((nf, m.nrows_pad), dtype=torch.bfloat16, device=dev)
    k.mf_split_w(W.data_ptr(), m.nrows_pad, nf, m.nrows_pad, Wh.data_ptr(), Wl.data_ptr(), s, True)
    ns = k.mf_backproject_b16_num_splits(m.ld, P, True)
    part = torch.zeros((ns, m.ld, nf), device=dev)
    os.environ["SART_MF_X3_DEPTH"] = "2"
    os.environ["SART_MF_X3_VT"] = "1"
    for abl in [int(v) for v in os.environ.get("PROBE_ABL", "0,1,2,4,3,5,6,7,0").split(",")]:
        os.environ["SART_MF_ABL"] = str(abl)
        med, best = timeit(lambda: k.mf_backproject_x3(m.A.data_ptr(), m.ld, P, Wh.data_ptr(), Wl.data_ptr(),
                                                       m.nrows_pad, ns, part.data_ptr(), s, nf), reps=7)
        print(json.dumps(dict(op="mf_backproject_x3", abl=abl, no_mfma=bool(abl & 1), no_split=bool(abl & 2),
                              no_w_lds=bool(abl & 4), nf=nf, P=P, V=V, nsplit=ns, ms=round(med, 4),
                              GBps=round(m.nbytes / med / 1e6, 1))), flush=True)
    # the register-W back-projection (k_mf_backproject_x3_reg: no LDS, no barrier) against the LDS kernel
    os.environ.pop("SART_MF_ABL", None)
    ref = None
    for bwd, depth in [tuple(v.split(":")) for v in os.environ.get(
            "PROBE_BWD", "lds:2,h16:2,lds:2,h16:2").split(";" if ";" in os.environ.get("PROBE_BWD", "") else ",")]:
        # "<variant>_vt2": two 64-voxel tiles per wave (SART_MF_X3_VT=2); "h16[+opts]": the f16-pair kernel
        name = bwd
        os.environ["SART_MF_X3_VT"] = "2" if bwd.endswith("_vt2") else "1"
        os.environ["SART_MF_X3_DEPTH"] = str(depth)
        nsv = k.mf_backproject_b16_num_splits(m.ld, P, True)  # m32 / vt 2: 128 voxels per wave, its own split count
        pv = torch.zeros((nsv, m.ld, nf), device=dev)
        if bwd.startswith("h16"):  # f16 pairs, three products (launch_mf_backproject_h16); "h16+ew,w1": SART_MF_H16
            os.environ["SART_MF_H16"] = bwd[4:]
            scratch = torch.zeros(max(nf, m.ld), dtype=torch.int32, device=dev)
            csc = torch.zeros(2 * m.ld, device=dev)
            k.mf_col_scales(m.A.data_ptr(), m.ld, m.nrows_pad, scratch.data_ptr(), csc.data_ptr(), s)
            w16 = torch.zeros((2, nf, m.nrows_pad), dtype=torch.int16, device=dev)
            inv = torch.zeros(nf, device=dev)
            k.mf_split_w16(W.data_ptr(), m.nrows_pad, nf, m.nrows_pad, w16[0].data_ptr(), w16[1].data_ptr(),
                           scratch.data_ptr(), 1.0, inv.data_ptr(), s)
            med, best = timeit(lambda: k.mf_backproject_h16(m.A.data_ptr(), m.ld, P, w16[0].data_ptr(), w16[1].data_ptr(),
                                                            m.nrows_pad, nsv, pv.data_ptr(), s, nf, 0, m.ld,
                                                            csc.data_ptr(), inv.data_ptr()), reps=7)
        else:
            med, best = timeit(lambda: k.mf_backproject_x3(m.A.data_ptr(), m.ld, P, Wh.data_ptr(), Wl.data_ptr(),
                                                           m.nrows_pad, nsv, pv.data_ptr(), s, nf), reps=7)
        out = pv.double().sum(0)
        if ref is None:
            ref = out
        rel = float((out - ref).norm() / ref.norm())
        print(json.dumps(dict(op="mf_backproject_x3", variant=name, depth=depth, nf=nf, P=P, V=V, nsplit=nsv,
                              ms=round(med, 4), GBps=round(m.nbytes / med / 1e6, 1),
                              rel_vs_first=rel, bitwise_equal_first=bool(rel == 0.0))), flush=True)
        del pv
    os.environ["SART_MF_X3_VT"] = "1"
    # the split-A forward (k_mf_forward_b16_lds<4, 3, 2, 1, float, true, ABL>: A staged through LDS, X in LDS)
    X = torch.rand((nf, m.ld), device=dev)
    Xh = torch.empty((nf, m.ld), dtype=torch.bfloat16, device=dev)
    Xl = torch.empty_like(Xh)
    k.mf_split_x(X.data_ptr(), nf * m.ld, Xh.data_ptr(), Xl.data_ptr(), s, True)
    nsf = k.mf_forward_num_splits(m.ld, m.nrows_pad)
    Fo = torch.zeros((nsf, m.nrows_pad, nf), device=dev)
    os.environ["SART_MF_X3_DEPTH"] = "3"
    os.environ["SART_MF_X3_FWD"] = "2,1,as"
    for abl in [int(v) for v in os.environ.get("PROBE_ABL", "0,1,2,4,3,5,6,7,0").split(",")]:
        os.environ["SART_MF_ABL"] = str(abl)
        med, best = timeit(lambda: k.mf_forward_x3(m.A.data_ptr(), m.ld, P, m.nrows_pad, Xh.data_ptr(), Xl.data_ptr(),
                                                   Fo.data_ptr(), nsf, s, nf), reps=7)
        print(json.dumps(dict(op="mf_forward_x3", abl=abl, no_mfma=bool(abl & 1), no_split=bool(abl & 2),
                              no_x_lds=bool(abl & 4), nf=nf, P=P, V=V, nsplit=nsf, ms=round(med, 4),
                              GBps=round(m.nbytes / med / 1e6, 1))), flush=True)
    for key in ("SART_MF_ABL", "SART_MF_X3_DEPTH", "SART_MF_X3_FWD", "SART_MF_X3_VT", "SART_MF_H16"):
        os.environ.pop(key, None)


if __name__ == "__main__":
    main()
