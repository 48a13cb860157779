"""Host view of the device-resident ``SartState`` (csrc/kernels/sart_common.hpp).

The reference keeps the iteration counter, the convergence metric and the status on the host and
synchronises for them every iteration (reference sartsolver_cuda.cpp:231-262). Here they live in a
128-byte device struct updated by ``k_decide``; the host reads it only between chunks of iterations.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

STATE_NBYTES = 128
_FMT = "<ddddiiiiiidii"  # up to `flags`; the rest is reserved
_SIZE = struct.calcsize(_FMT)

SUCCESS = 0
MAX_ITERATIONS_EXCEEDED = -1
RUNNING = -2


@dataclass
class SartStateView:
    G: float
    conv_prev: float
    conv_last: float
    F_last: float
    sweep: int
    done: int
    status: int
    iterations: int
    max_iter: int
    error: int
    tol: float
    epoch: int

    @classmethod
    def from_bytes(cls, raw: bytes) -> "SartStateView":
        vals = struct.unpack(_FMT, raw[:_SIZE])
        return cls(*vals[:12])


def new_state(device):
    import torch

    return torch.zeros(STATE_NBYTES, dtype=torch.uint8, device=device)


def read_state(state_tensor) -> SartStateView:
    return SartStateView.from_bytes(state_tensor.cpu().numpy().tobytes())
