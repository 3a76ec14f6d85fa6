"""Multi-GPU sharding of the verify / MSM path: one process per GPU,
torch.distributed ("nccl" = RCCL on ROCm) for the few bytes that cross GPUs.

* Batch verify (BASELINE configs[1], [4]): proofs are independent, so each rank verifies a
  contiguous shard of the batch and nothing crosses GPUs on the data path.  Verdicts are
  gathered afterwards (``gather_verdicts``: B bytes over xGMI).
* One large MSM (configs[2] on N GPUs): the reference's MSM reduction is the canonical
  pairwise tree (cuda_bulletproof_kernels.cu:45-115).  With shards of m = 2^j
  consecutive points starting at multiples of m, levels 1..m/2 of the tree stay inside a
  shard and the remaining levels are the canonical tree over the shard roots in index
  order, so per-rank MSMs + one all_gather of 128-byte roots + a tree over them on every
  rank is bit-exact with the single-GPU MSM.  RCCL has no point-add reduction op, hence
  all_gather + tree rather than all_reduce.

* One large Pippenger MSM (the labelled alternative, BASELINE configs[2]'s window 12): its windows
  are independent until the final Horner chain, so each rank forms the window sums S_w of a
  contiguous window range over ALL points, the 128-byte sums meet in one all_gather (RCCL cannot
  add points, so no all_reduce), and every rank runs the Horner over the W sums: bit-exact with
  the single-GPU ``msm_pippenger``, whose windows are formed the same way.

The compute callables default to the HIP kernels (``msm`` / ``point_tree`` of this package);
the CPU gloo tests (tests/test_shard.py) pass CPU checkers in their place to test the host logic.
"""
import torch
import torch.distributed as dist


def shard_bounds(total, world, rank):
    """Contiguous shard [lo, hi) of `total` independent items for `rank` (sizes differ by <= 1)."""
    q, r = divmod(int(total), int(world))
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def msm_shard_plan(n, world):
    """(m, K): shard size m (power of two, m * world >= n) and the number K = ceil(n / m) of
    non-empty shards.  Rank k < K owns points [k m, min(n, (k+1) m))."""
    n, world = int(n), int(world)
    if n <= 0:
        return 1, 0
    per = -(-n // world)
    m = 1 << (per - 1).bit_length()
    return m, -(-n // m)


def msm_shard_bounds(n, world, rank):
    m, K = msm_shard_plan(n, world)
    lo = min(n, rank * m)
    return lo, min(n, lo + m) if rank < K else lo


def _hip_msm(scalars, points):
    from . import msm
    out = torch.zeros(16, dtype=torch.int64, device=points.device)
    msm(out, scalars, points)
    return out


def _hip_tree(points):
    from . import point_tree
    out = torch.zeros(16, dtype=torch.int64, device=points.device)
    point_tree(out, points)
    return out


def sharded_msm(scalars, points, n_total, group=None, local_msm=None, tree=None):
    """Canonical-tree MSM of `n_total` points spread over the ranks of `group`.

    scalars (k,4) / points (k,16): this rank's shard, rows msm_shard_bounds(n_total, world, rank)
    of the full input (k may be 0).  Returns the (16,) int64 result on every rank, bit-exact
    with ``msm`` over the whole input on one GPU.
    """
    local_msm = local_msm or _hip_msm
    tree = tree or _hip_tree
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    m, K = msm_shard_plan(n_total, world)
    lo, hi = msm_shard_bounds(n_total, world, rank)
    if points.shape[0] != hi - lo or scalars.shape[0] != hi - lo:
        raise ValueError(f"rank {rank}: shard has {points.shape[0]} points, plan expects {hi - lo}")
    if K == 0:
        raise ValueError("empty MSM")
    root = local_msm(scalars, points) if hi > lo else torch.zeros(16, dtype=torch.int64, device=points.device)
    if world == 1:
        return root
    parts = [torch.empty(16, dtype=torch.int64, device=points.device) for _ in range(world)]
    dist.all_gather(parts, root.contiguous(), group=group)
    roots = torch.stack(parts)
    return tree(roots[:K].contiguous()) if K > 1 else roots[0].clone()


def gather_verdicts(ok_local, total, group=None):
    """All ranks' verdict bytes (shard_bounds layout) -> (total,) uint8 on every rank."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    cap = shard_bounds(total, world, 0)[1]
    lo, hi = shard_bounds(total, world, rank)
    if ok_local.shape[0] != hi - lo:
        raise ValueError("verdict shard does not match shard_bounds")
    buf = torch.zeros(cap, dtype=torch.uint8, device=ok_local.device)
    buf[:hi - lo] = ok_local
    allb = [torch.empty(cap, dtype=torch.uint8, device=ok_local.device) for _ in range(world)]
    dist.all_gather(allb, buf, group=group)
    parts = [allb[r][:shard_bounds(total, world, r)[1] - shard_bounds(total, world, r)[0]] for r in range(world)]
    return torch.cat(parts)


def pippenger_window_bounds(window_bits, world, rank):
    """Contiguous window range [w0, w1) of rank `rank` (W = ceil(256 / window_bits) windows).

    Windows are split by cost, not count: a narrow top window (fewer than c/2 bits: 4 at c = 12,
    3 for the 255-bit config-3 scalars) has few, deep buckets whose trees run latency-bound tail
    steps, and costs about three ordinary windows (2^20 points, c = 12, one MI355X:
    tools/pip_shard_probe.py).  Window w goes to rank floor(start_w * world / total), start_w =
    the cost of the windows below it, so the ranges are contiguous and cover every window."""
    c = int(window_bits)
    W = (256 + c - 1) // c
    top_bits = 256 - c * (W - 1)
    cost = [1] * (W - 1) + [3 if 2 * top_bits < c else 1]
    total = sum(cost)
    owner, start = [], 0
    for w in range(W):
        owner.append(min(world - 1, start * world // total))
        start += cost[w]
    ws = [w for w in range(W) if owner[w] == rank]
    if ws:
        return ws[0], ws[-1] + 1
    lo = next((w for w in range(W) if owner[w] > rank), W)   # empty range at its place in the order
    return lo, lo


def _hip_windows(scalars, points, w0, w1, window_bits):
    from . import msm_pippenger_windows, pippenger_num_windows
    W = pippenger_num_windows(window_bits)
    Sw = torch.zeros(W, 16, dtype=torch.int64, device=points.device)
    msm_pippenger_windows(Sw, scalars, points, w0, w1, window_bits)
    return Sw[w0:w1]


def _hip_horner(Sw, window_bits):
    from . import msm_pippenger_horner
    out = torch.zeros(16, dtype=torch.int64, device=Sw.device)
    msm_pippenger_horner(out, Sw.contiguous(), window_bits)
    return out


def sharded_msm_pippenger(scalars, points, window_bits=12, group=None, windows=None, horner=None):
    """Pippenger MSM of all n points with its windows split over the ranks of `group`.

    Every rank holds all scalars (n,4) and points (n,16).  Rank r forms the window sums of
    pippenger_window_bounds(window_bits, world, r); one all_gather of (largest range, 16)
    int64 rows per rank brings all W sums to every rank; each runs the Horner chain.  Returns
    the (16,) int64 result on every rank, bit-exact with ``msm_pippenger`` on one GPU.
    `windows(scalars, points, w0, w1, c) -> (w1 - w0, 16)` and `horner(Sw, c) -> (16,)` default
    to the HIP kernels (the CPU tests pass their own checkers).
    """
    windows = windows or _hip_windows
    horner = horner or _hip_horner
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    W = (256 + int(window_bits) - 1) // int(window_bits)
    if points.shape[0] == 0 or scalars.shape[0] != points.shape[0]:
        raise ValueError("sharded_msm_pippenger: need one scalar per point and n > 0")
    w0, w1 = pippenger_window_bounds(window_bits, world, rank)
    if world == 1:
        return horner(windows(scalars, points, 0, W, window_bits), window_bits)
    spans = [pippenger_window_bounds(window_bits, world, r) for r in range(world)]
    cap = max(b - a for a, b in spans)
    buf = torch.zeros(cap, 16, dtype=torch.int64, device=points.device)
    if w1 > w0:
        buf[:w1 - w0] = windows(scalars, points, w0, w1, window_bits)
    parts = [torch.empty(cap, 16, dtype=torch.int64, device=points.device) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    Sw = torch.cat([parts[r][:b - a] for r, (a, b) in enumerate(spans)])
    return horner(Sw.contiguous(), window_bits)
