"""Per-lane digests of the step tensors on the device, for the every-lane
parity tests at the bench sizes.

Test infrastructure: the observation / information-state rows of every lane
are reduced on the GPU to the two linear hashes oracle/coup_oracle.c's window
driver computes on the host (oc_window_args: h_j = sum_i bits(x_i) * w_j[i],
w_j < 2^18 from oracle.hash_weights), so the 2^20-lane tensors are checked on
every lane without copying 822 MB per step to the host.  Exact in int64: at
most 2 x 2492 terms below 2^32 * 2^18.  A single wrong float always changes
both hashes (every weight is non-zero); two independent weight rows make a
multi-float coincidence ~2^-36 per lane."""
import numpy as np
import torch

from oracle import oracle


def tensor_hash(x, chunk_elems=1 << 28):
    """x: float32 [B, ...] tensor on any device (the [B][2][98] or
    [B][2][2492] rows of one step) -> uint64 [B, 2] numpy."""
    B = x.shape[0]
    flat = x.reshape(B, -1)
    L = flat.shape[1]
    w = torch.from_numpy(oracle.hash_weights(L).astype(np.int64)).to(x.device)
    out = torch.empty(B, 2, dtype=torch.int64, device=x.device)
    step = max(1, chunk_elems // L)
    for lo in range(0, B, step):
        bits = flat[lo:lo + step].contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        out[lo:lo + step, 0] = (bits * w[0]).sum(1)
        out[lo:lo + step, 1] = (bits * w[1]).sum(1)
        del bits
    return out.cpu().numpy().view(np.uint64)


def first_mismatch(got, want, what):
    """None if equal, else a message naming the first differing lane."""
    got, want = np.asarray(got), np.asarray(want)
    if got.shape != want.shape:
        return f"{what}: shape {got.shape} != {want.shape}"
    bad = np.nonzero((got != want).reshape(got.shape[0], -1).any(1))[0]
    if bad.size == 0:
        return None
    i = int(bad[0])
    return f"{what}: {bad.size} of {got.shape[0]} lanes differ, first lane {i}: {got[i]!r} != {want[i]!r}"


def assert_lanes_equal(got, want, what):
    msg = first_mismatch(got, want, what)
    assert msg is None, msg
