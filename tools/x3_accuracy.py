#!/usr/bin/env python3
"""Accuracy of the multi-frame projections per operand path against fp64: fp32 MFMA (multiframe.hip), split-A bf16
MFMA (fp32 A split in registers, multiframe_bf16.hip) on the same fp32 shard. One JSON line per op and path:
norm-relative and max relative error of F = A X^T and B = A^T W."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mpi_cuda_sartsolver_amd.models.rtm import DenseRTM  # noqa: E402
from mpi_cuda_sartsolver_amd.ops import hip  # noqa: E402


def main():
    k = hip()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    P, V, nf = 2048, 4096, 32
    rng = np.random.default_rng(3)
    A = rng.random((P, V), dtype=np.float32)
    m = DenseRTM.from_dense(A, device=dev)
    Ad = A.astype(np.float64)
    X = rng.random((nf, V)).astype(np.float32)
    W = (rng.random((P, nf)) - 0.5).astype(np.float32)
    F_ref = Ad @ X.T.astype(np.float64)
    B_ref = Ad.T @ W.astype(np.float64)

    def err(name, op, got, ref):
        d = got - ref
        print(json.dumps(dict(op=op, path=name, rel_norm=float(np.linalg.norm(d) / np.linalg.norm(ref)),
                              max_rel=float(np.max(np.abs(d) / np.maximum(np.abs(ref), 1e-30))),
                              mean_rel=float(np.mean(d / np.where(ref == 0, 1, ref))))), flush=True)

    Xd = torch.zeros((nf, m.ld), device=dev)
    Xd[:, :V] = torch.from_numpy(X)
    Wd = torch.zeros((m.nrows_pad, nf), device=dev)
    Wd[:P] = torch.from_numpy(np.ascontiguousarray(W.reshape(P, nf // 16, 16).transpose(0, 2, 1).reshape(P, nf)))
    nsf = k.mf_forward_num_splits(m.ld, m.nrows_pad)
    Fo = torch.zeros((nsf, m.nrows_pad, nf), device=dev)
    k.mf_forward(m.A.data_ptr(), m.ld, P, m.nrows_pad, Xd.data_ptr(), m.ld, Fo.data_ptr(), nsf, s, nf)
    ns = k.mf_backproject_num_splits(m.ld, P)
    part = torch.zeros((ns, m.ld, nf), device=dev)
    k.mf_backproject(m.A.data_ptr(), m.ld, P, Wd.data_ptr(), ns, part.data_ptr(), s, nf)
    torch.cuda.synchronize()
    err("fp32", "forward", Fo.sum(0)[:P].double().cpu().numpy(), F_ref)
    err("fp32", "backproject", part.sum(0)[:V].double().cpu().numpy(), B_ref)  # natural frame order

    Xh = torch.empty((nf, m.ld), dtype=torch.bfloat16, device=dev)
    Xl = torch.empty_like(Xh)
    k.mf_split_x(Xd.data_ptr(), nf * m.ld, Xh.data_ptr(), Xl.data_ptr(), s, True)
    Fo.zero_()
    k.mf_forward_x3(m.A.data_ptr(), m.ld, P, m.nrows_pad, Xh.data_ptr(), Xl.data_ptr(), Fo.data_ptr(), nsf, s, nf)
    Wh = torch.zeros((2, nf, m.nrows_pad), dtype=torch.bfloat16, device=dev)  # hi, mid
    Wl = torch.zeros((nf, m.nrows_pad), dtype=torch.bfloat16, device=dev)
    k.mf_split_w(Wd.data_ptr(), m.nrows_pad, nf, m.nrows_pad, Wh.data_ptr(), Wl.data_ptr(), s, True)
    nsb = k.mf_backproject_b16_num_splits(m.ld, P, True)
    part = torch.zeros((nsb, m.ld, nf), device=dev)
    k.mf_backproject_x3(m.A.data_ptr(), m.ld, P, Wh.data_ptr(), Wl.data_ptr(), m.nrows_pad, nsb, part.data_ptr(), s, nf)
    torch.cuda.synchronize()
    err("x3", "forward", Fo.sum(0)[:P].double().cpu().numpy(), F_ref)
    err("x3", "backproject", part.sum(0)[:V].double().cpu().numpy(), B_ref)
    # sensitivity: without the lo planes (hi only) the error would be
    Fo.zero_()
    k.mf_forward_x3(m.A.data_ptr(), m.ld, P, m.nrows_pad, Xh.data_ptr(), torch.zeros_like(Xl).data_ptr(),
                    Fo.data_ptr(), nsf, s, nf)
    part.zero_()
    k.mf_backproject_x3(m.A.data_ptr(), m.ld, P, Wh.data_ptr(), torch.zeros_like(Wl).data_ptr(), m.nrows_pad, nsb,
                        part.data_ptr(), s, nf)
    torch.cuda.synchronize()
    err("x3 without X/W lo", "forward", Fo.sum(0)[:P].double().cpu().numpy(), F_ref)
    err("x3 without X/W lo", "backproject", part.sum(0)[:V].double().cpu().numpy(), B_ref)


if __name__ == "__main__":
    main()
