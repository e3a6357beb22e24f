"""lachain_amd/shard.py — how the batch path is split over GPUs (one process per GPU, torch.distributed).

SURVEY.md §8e: share verifications are independent, so batches are partitioned by ciphertext (TPKE) or by
round (threshold signatures), keeping every share that pairs with the same H / W / message on one GPU (its
line sets are computed once there).  No data-path collective is needed for them; the per-rank accept bitmaps
are gathered only when a caller wants the whole bitmap on one rank.  The G1 MSM is the one path with a real
exchange step: each rank reduces its slice of points to one Jacobian partial (144 B), the partials are
all-gathered over RCCL (xGMI) and summed on the GPU.

The helpers take the collective module (`torch.distributed`) and tensors as arguments, so the same code runs
over RCCL on MI355X and over gloo on CPU (tests/test_multirank.py).
"""


def block_range(n_units, rank, world):
    """Contiguous block [lo, hi) of n_units owned by `rank` (sizes differ by at most one)."""
    base, extra = divmod(n_units, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def tpke_shard(ct_idx, n_cts, rank, world):
    """Shares of the ciphertexts [lo, hi) owned by `rank`: (lo, hi, share indices).  ct_idx is the per-share
    ciphertext index (numpy array); shares keep their batch order."""
    import numpy as np
    lo, hi = block_range(n_cts, rank, world)
    sel = np.nonzero((ct_idx >= lo) & (ct_idx < hi))[0]
    return lo, hi, sel


def _host_comm(dist, t):
    """gloo moves host tensors only: a device tensor is exchanged through host memory under a non-RCCL backend"""
    return t.is_cuda and dist.get_backend() != "nccl"


def all_gather_fixed(dist, local, world):
    """All-gather of equal-sized 1-D uint8 tensors -> one tensor of world * len(local) bytes (rank order)."""
    import torch
    out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
    if world == 1:
        out.copy_(local)
    elif _host_comm(dist, local):
        host = torch.empty(world * local.numel(), dtype=local.dtype)
        dist.all_gather_into_tensor(host, local.cpu())
        out.copy_(host)
    else:
        dist.all_gather_into_tensor(out, local)
    return out


def max_time_sum(dist, torch, dev, elapsed, *counts):
    """The bench's cross-rank reduction: [max over ranks of elapsed (a job takes as long as its slowest rank),
    sum over ranks of each count].  Plain floats at world size 1 or without a process group."""
    vals = [float(elapsed)] + [float(c) for c in counts]
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return vals
    cd = dev if dist.get_backend() == "nccl" else "cpu"
    tm = torch.tensor(vals[:1], dtype=torch.float64, device=cd)
    ts = torch.tensor(vals[1:] + [0.0], dtype=torch.float64, device=cd)
    dist.all_reduce(tm, op=dist.ReduceOp.MAX)
    dist.all_reduce(ts, op=dist.ReduceOp.SUM)
    return [float(tm[0])] + [float(x) for x in ts.tolist()[:len(counts)]]


def gather_bitmaps(dist, local_bits, world):
    """All-gather per-rank accept bitmaps of different lengths (uint8, one byte per share); returns the list
    of per-rank bitmaps (as numpy arrays) in rank order."""
    import torch
    n = torch.tensor([local_bits.numel()], dtype=torch.int64, device=local_bits.device)
    sizes = all_gather_fixed(dist, n.view(torch.uint8), world).view(torch.int64).tolist()
    m = max(sizes)
    padded = torch.zeros(m, dtype=torch.uint8, device=local_bits.device)
    padded[:local_bits.numel()] = local_bits
    allb = all_gather_fixed(dist, padded, world).cpu().numpy()
    return [allb[r * m:r * m + sizes[r]] for r in range(world)]


def msm_combine(dist, local_partial, world, sum_partials):
    """MSM exchange step: all-gather the per-rank partials (fixed-size byte tensors) and reduce them with
    sum_partials(gathered_tensor, world) (lcb_g1_jac_sum_dev on the GPU)."""
    return sum_partials(all_gather_fixed(dist, local_partial, world), world)
