#!/usr/bin/env python3
"""Split-count probe of the MFMA back-projection (partials [splits][ld][nf] are summed by k_mf_collect):
kernel time per split count at the default tiling, 64k x 64k. One JSON line per measurement."""
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
    P = V = 65536
    m = DenseRTM.synthetic(P, V, 0, seed=1, device=dev)
    for nf in (16, 32, 64):
        W = torch.rand((m.nrows_pad, nf), device=dev)
        part = torch.zeros((32, m.ld, nf), device=dev)
        for ns in (2, 4, 8, 16, 32):
            med, _ = timeit(lambda: k.mf_backproject(m.A.data_ptr(), m.ld, P, W.data_ptr(), ns, part.data_ptr(), s, nf),
                            reps=7)
            print(json.dumps(dict(op="mf_backproject", nf=nf, nsplit=ns, default=k.mf_backproject_num_splits(m.ld, P),
                                  ms=round(med, 4), TFLOPs=round(2 * nf * P * V / med / 1e9, 2))), flush=True)
        del W, part
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
