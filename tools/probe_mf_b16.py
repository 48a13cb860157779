#!/usr/bin/env python3
"""bf16 multi-frame projection probe: k_mf_forward_b16 / k_mf_backproject_b16 time per batch width, ring depth and
tile (SART_MF_DEPTH, SART_MF_B16_FWD = "RT,KB", SART_MF_B16_VT) on a synthetic bf16 shard (default 65536 x 65536).
One JSON line per measurement."""
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
    m = DenseRTM.synthetic(P, V, 0, seed=1, device=dev, storage="bf16")
    nbytes = m.nbytes
    nfs = [int(v) for v in os.environ.get("PROBE_NF", "16,32,64").split(",")]
    fwd_tiles = os.environ.get("PROBE_FWD", "4,1;2,2;4,2;8,1;4,1,lds;4,2,lds;8,1,lds;2,2,lds").split(";")
    for nf in nfs:
        Xh = torch.rand((nf, m.ld), device=dev).bfloat16()
        Xl = (torch.rand((nf, m.ld), device=dev) * 1e-3).bfloat16()
        Fo = torch.zeros((16, m.nrows_pad, nf), device=dev)
        Wh = torch.rand((nf, m.nrows_pad), device=dev).bfloat16()
        Wl = (torch.rand((nf, m.nrows_pad), device=dev) * 1e-3).bfloat16()
        part = torch.zeros((64, m.ld, nf), device=dev)
        for depth in [int(v) for v in os.environ.get("PROBE_DEPTH", "1,2,3").split(",")]:
            os.environ["SART_MF_DEPTH"] = str(depth)
            for tile in fwd_tiles:
                os.environ["SART_MF_B16_FWD"] = tile
                nsf = k.mf_forward_num_splits(m.ld, m.nrows_pad)
                med, best = timeit(lambda: k.mf_forward_b16(m.A.data_ptr(), m.ld, P, m.nrows_pad, Xh.data_ptr(),
                                                            Xl.data_ptr(), Fo.data_ptr(), nsf, s, nf), reps=5)
                print(json.dumps(dict(op="mf_forward_b16", nf=nf, depth=depth, tile=tile, nsplit=nsf, P=P, V=V,
                                      ms=round(med, 4), GBps=round(nbytes / med / 1e6, 1),
                                      TFLOPs=round(4 * nf * P * V / med / 1e9, 1))), flush=True)
            for vt in (os.environ.get("PROBE_VT", "1,reg;2,reg;1,lds;2,lds").split(";")
                       if os.environ.get("PROBE_BWD", "1") == "1" else ()):
                os.environ["SART_MF_B16_VT"] = str(vt)
                ns = k.mf_backproject_b16_num_splits(m.ld, P)
                assert ns <= 64
                med, best = timeit(lambda: k.mf_backproject_b16(m.A.data_ptr(), m.ld, P, Wh.data_ptr(), Wl.data_ptr(),
                                                                m.nrows_pad, ns, part.data_ptr(), s, nf), reps=5)
                print(json.dumps(dict(op="mf_backproject_b16", nf=nf, depth=depth, vt=vt, nsplit=ns, P=P, V=V,
                                      ms=round(med, 4), GBps=round(nbytes / med / 1e6, 1),
                                      TFLOPs=round(4 * nf * P * V / med / 1e9, 1))), flush=True)
        for key in ("SART_MF_DEPTH", "SART_MF_B16_FWD", "SART_MF_B16_VT"):
            os.environ.pop(key, None)
        del Xh, Xl, Fo, Wh, Wl, part
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
