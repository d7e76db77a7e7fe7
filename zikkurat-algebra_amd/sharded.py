"""Multi-GPU MSM: shard the pairs by contiguous chunk, one exchange of partial sums.

The reference is single-device (bls12_381_G1_proj.c:630-644).  An MSM is a
group sum, so it partitions exactly: rank r computes S_r = sum_{i in chunk r} k_i P_i on its own
GPU, the G partial points (3*NP u64 each, 96-144 B) are all-gathered, and every rank adds them
in rank order.  The affine result is identical for any split, so the sharded answer is
bit-exact against the single-device one.  The payload is tiny: the exchange is latency-bound,
not link-bandwidth-bound.  RCCL has no elliptic-curve reduction operator, so "reduce" =
all-gather + local adds.

On GPUs the exchange is the library's own (``LibComm``: ncclAllGather from /opt/rocm's RCCL on
the library's stream, ``zkg_g1_msm_device_sharded``), so a process holds ONE HIP runtime and no
torch.  The rendezvous is a file: rank 0 writes the 128-byte RCCL unique id, the other ranks
read it (``comm_init``).  ``allgather_partials`` (torch.distributed) remains for the CPU gloo
tests, which rehearse the same shard / combine logic without a GPU.
"""
import ctypes
import os
import tempfile
import time

import numpy as np

import zkalgebra as zk

COMM_ID_BYTES = 128


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
    """all-gather one projective point (u64 words) from every rank over torch.distributed, rank
    order (CPU gloo rehearsals; the GPU path uses LibComm)."""
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


# ----------------------------------------------------------------------------- library communicator

def rendezvous_path():
    """file through which rank 0 hands the RCCL unique id to the other ranks of one launch.
    The key defaults to (launcher pid, MASTER_PORT): every rank of a torchrun launch is a child
    of the same agent process, and the port separates concurrent launches.  Launchers whose ranks
    do not share a parent process (mpirun, srun, a shell loop) must set ZKG_RDZV_KEY to one value
    per launch on every rank (and ZKG_RDZV_DIR to a directory every rank sees); bench.py's own
    launcher sets both ZKG_RDZV_KEY and ZKG_RDZV_NONCE."""
    d = os.environ.get("ZKG_RDZV_DIR") or tempfile.gettempdir()
    key = os.environ.get("ZKG_RDZV_KEY")
    if not key:
        if "TORCHELASTIC_RUN_ID" not in os.environ and int(os.environ.get("WORLD_SIZE", "1")) > 1:
            raise RuntimeError("multi-rank run without torchrun: set ZKG_RDZV_KEY (one value per launch, the same "
                               "on every rank) so the ranks find one rendezvous file")
        key = f"{os.getppid()}_{os.environ.get('MASTER_PORT', '0')}"
    return os.path.join(d, f"zkg_rdzv_{key}.id")


def rendezvous_nonce():
    """per-launch tag written after the id: a rank accepts only an id file carrying its own
    launch's tag, so a stale file left by an earlier launch with the same key is never used.
    ZKG_RDZV_NONCE (bench.py's launcher), else torchrun's run id and restart count -- the same on
    every node of a launch (each node's elastic agent is a different process, so nothing per-process
    may enter it: ADVICE r05); empty (no check) otherwise.  With torchrun's default run id ("none")
    the tag does not tell launches apart; rank 0's removal of the old file and the per-launch key
    then carry that."""
    n = os.environ.get("ZKG_RDZV_NONCE")
    if n:
        return n.encode()
    if "TORCHELASTIC_RUN_ID" in os.environ:
        return f"{os.environ['TORCHELASTIC_RUN_ID']}:{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}".encode()
    return b""


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc})")


class LibComm:
    """The library's RCCL communicator (zkg_comm_*), one per process: barrier, max over ranks,
    sharded device-resident MSM.  Construct after zkg_set_device."""

    def __init__(self, rank, world, timeout=600.0):
        lib = zk.load()
        self.rank, self.world = rank, world
        uid = ctypes.create_string_buffer(COMM_ID_BYTES)
        path = rendezvous_path()
        nonce = rendezvous_nonce()
        try:
            if rank == 0:
                try:
                    os.unlink(path)  # a stale id of an earlier launch with this key
                except OSError:
                    pass
                _check(lib.zkg_comm_unique_id(uid), "zkg_comm_unique_id")
                tmp = f"{path}.{os.getpid()}.tmp"
                with open(tmp, "wb") as f:
                    f.write(uid.raw[:COMM_ID_BYTES] + nonce)
                os.replace(tmp, path)  # atomic: readers see the whole id or nothing
            else:
                t0 = time.time()
                while True:
                    try:
                        with open(path, "rb") as f:
                            raw = f.read()
                        if len(raw) >= COMM_ID_BYTES and raw[COMM_ID_BYTES:] == nonce:
                            break
                    except FileNotFoundError:
                        pass
                    if time.time() - t0 > timeout:
                        raise TimeoutError(f"rank {rank}: no RCCL unique id of this launch at {path} after "
                                           f"{timeout:.0f} s")
                    time.sleep(0.01)
                ctypes.memmove(uid, raw[:COMM_ID_BYTES], COMM_ID_BYTES)
            _check(lib.zkg_comm_init(rank, world, uid), "zkg_comm_init")
        finally:
            # ncclCommInitRank is collective: once rank 0 returns, every rank has read the id (and if
            # rank 0 failed, its id must not be picked up by anyone later)
            if rank == 0:
                try:
                    os.unlink(path)
                except OSError:
                    pass

    def barrier(self):
        _check(zk.load().zkg_comm_barrier(), "zkg_comm_barrier")

    def max(self, x):
        v = ctypes.c_double(float(x))
        _check(zk.load().zkg_comm_max_f64(ctypes.byref(v)), "zkg_comm_max_f64")
        return v.value

    def allgather(self, arr):
        """host array (same shape on every rank) -> stacked array of every rank's copy"""
        a = np.ascontiguousarray(arr)
        out = np.empty((self.world,) + a.shape, dtype=a.dtype)
        _check(zk.load().zkg_comm_allgather(a.ctypes.data, out.ctypes.data, a.nbytes), "zkg_comm_allgather")
        return out

    def sum_partials(self, curve, partials):
        """(count, 3 NP) projective partials of this rank -> normalised sum over every rank's"""
        p = np.ascontiguousarray(partials, dtype=np.uint64).reshape(-1, 3 * zk.NLIMBS_P[curve])
        out = np.zeros(3 * zk.NLIMBS_P[curve], dtype=np.uint64)
        _check(zk.load().zkg_g1_comm_sum_partials(zk.CURVE_ID[curve], zk._p(p), p.shape[0], zk._p(out)),
               "zkg_g1_comm_sum_partials")
        return out

    def msm_device_sharded(self, curve, n_local, d_scalars, d_points, mont=True, window=0, nlimbs=4,
                           local_shards=1):
        """this rank's chunk (device buffers) -> normalised projective MSM of every rank's chunk"""
        out = np.zeros(3 * zk.NLIMBS_P[curve], dtype=np.uint64)
        _check(zk.load().zkg_g1_msm_device_sharded(zk.CURVE_ID[curve], n_local, d_scalars.ptr, nlimbs,
                                                   1 if mont else 0, d_points.ptr, window, local_shards,
                                                   zk._p(out)), "zkg_g1_msm_device_sharded")
        return out

    def close(self):
        _check(zk.load().zkg_comm_destroy(), "zkg_comm_destroy")
