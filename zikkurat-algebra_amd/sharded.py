"""Multi-GPU MSM: shard the pairs by contiguous chunk, one exchange of partial sums.

The reference is single-device.  An MSM is a group sum, so it
partitions exactly: rank r computes S_r = sum_{i in chunk r} k_i P_i on its own GPU, the
G partial points (3*NP u64 each, 96-144 B) are all-gathered over RCCL (torch.distributed
"nccl" backend = RCCL on ROCm, over xGMI), and every rank adds them in rank order on the
host.  The affine result is identical for any split, so the sharded answer is bit-exact
against the single-device one.  The payload is tiny: the exchange is latency-bound, not
link-bandwidth-bound.

RCCL has no elliptic-curve reduction operator, so "reduce" = all-gather + local adds.
"""
import numpy as np

import zkalgebra as zk


def shard_range(n_total, rank, world):
    """contiguous chunk [lo, hi) of rank `rank`"""
    lo = n_total * rank // world
    hi = n_total * (rank + 1) // world
    return lo, hi


def combine_partials(curve, partials):
    """rank-ordered list of projective partials -> (projective sum, affine sum)"""
    acc = np.ascontiguousarray(partials[0])
    for p in partials[1:]:
        acc = zk.g1_add(curve, acc, np.ascontiguousarray(p))
    return zk.g1_normalize(curve, acc), zk.g1_to_affine(curve, acc)


def allgather_partials(partial, device=None):
    """all-gather one projective point (u64 words) from every rank, rank order."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    words = partial.shape[0]
    t = torch.from_numpy(np.ascontiguousarray(partial).view(np.int64).copy())
    if device is not None:
        t = t.to(device)
    out = torch.empty(world * words, dtype=torch.int64, device=t.device)
    dist.all_gather_into_tensor(out, t)
    host = out.cpu().numpy().view(np.uint64)
    return [host[r * words:(r + 1) * words] for r in range(world)]
