#!/usr/bin/env python3
"""Forward X-plane layout probe: the split-A (fp32 A) and bf16 64-frame forwards with frame-major X planes
([nf][ld]: a step's X tile is nf 64-byte pieces ld * 2 bytes apart) against blocked planes ([ld / 32][nf][32]: one
contiguous 4 KiB per plane and step), over the column-split count. Outputs must agree bit for bit (same k order,
same MFMAs). Shapes: argv (default 65536x65536 16384x262144). One JSON line per (shape, storage, nsplit, layout)."""
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
    nf = 64
    for shape in (sys.argv[1:] or ["65536x65536", "16384x262144"]):
        P, V = (int(v) for v in shape.split("x"))
        for storage in os.environ.get("PROBE_STORAGE", "fp32,bf16").split(","):
            m = DenseRTM.synthetic(P, V, 0, seed=1, device=dev, storage=storage)
            a32 = storage == "fp32"
            X = torch.rand((nf, m.ld), device=dev)
            planes = {}
            for blk in (False, True):
                Xh = torch.empty((nf, m.ld), dtype=torch.bfloat16, device=dev)
                Xl = torch.empty_like(Xh)
                k.mf_split_x(X.data_ptr(), nf * m.ld, Xh.data_ptr(), Xl.data_ptr(), s, a32, m.ld if blk else 0)
                planes[blk] = (Xh, Xl)
            nsf0 = k.mf_forward_num_splits(m.ld, m.nrows_pad)
            fwd = k.mf_forward_x3 if a32 else k.mf_forward_b16
            for nsf in ([] if os.environ.get("PROBE_TILES") else sorted({nsf0, 1, 2, 4, 8, 16} & set(range(1, 4 * nsf0 + 1)) | {nsf0})):
                Fo = {}
                for blk in (False, True, False, True):
                    Xh, Xl = planes[blk]
                    out = torch.zeros((nsf, m.nrows_pad, nf), device=dev)
                    med, _ = timeit(lambda: fwd(m.A.data_ptr(), m.ld, P, m.nrows_pad, Xh.data_ptr(), Xl.data_ptr(),
                                                out.data_ptr(), nsf, s, nf, blk), reps=7)
                    Fo.setdefault(blk, out)
                    print(json.dumps(dict(op="mf_forward_x3" if a32 else "mf_forward_b16", P=P, V=V, nf=nf,
                                          nsplit=nsf, default_nsplit=nsf == nsf0, xblk=blk, ms=round(med, 4),
                                          GBps=round(m.nbytes / med / 1e6, 1),
                                          bitwise_equal=bool(torch.equal(Fo[False], out)))), flush=True)
            # forward tiles / ring depths on blocked planes (PROBE_TILES="RT,KB[,as]:depth;..."), default split count
            tiles = os.environ.get("PROBE_TILES", "")
            tenv = "SART_MF_X3_FWD" if a32 else "SART_MF_B16_FWD"
            denv = "SART_MF_X3_DEPTH" if a32 else "SART_MF_DEPTH"
            ref = None
            for spec in [t for t in tiles.split(";") if t]:
                tile, depth = spec.split(":")
                os.environ[tenv], os.environ[denv] = tile, depth
                Xh, Xl = planes[True]
                out = torch.zeros((nsf0, m.nrows_pad, nf), device=dev)
                med, _ = timeit(lambda: fwd(m.A.data_ptr(), m.ld, P, m.nrows_pad, Xh.data_ptr(), Xl.data_ptr(),
                                            out.data_ptr(), nsf0, s, nf, True), reps=7)
                ref = out if ref is None else ref
                print(json.dumps(dict(op="mf_forward_x3" if a32 else "mf_forward_b16", P=P, V=V, nf=nf, nsplit=nsf0,
                                      xblk=True, tile=tile, depth=int(depth), ms=round(med, 4),
                                      GBps=round(m.nbytes / med / 1e6, 1),
                                      bitwise_equal_first=bool(torch.equal(ref, out)))), flush=True)
            for key in (tenv, denv):
                os.environ.pop(key, None)
            del m, X, planes
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
