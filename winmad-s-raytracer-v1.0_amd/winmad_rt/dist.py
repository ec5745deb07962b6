"""One process per GPU: how the BDPT / PT renders shard, and the single
collective step they have.

The reference renders a frame in one process (SurfaceIntegrator::render loops
over iterations / samples, surfaceIntegrator.cpp and bidirPathTracing.cpp:
BidirPathTracing::render); every iteration (BDPT) or sample (PT) is an
independent pass over the frame, and the counter RNG makes each one a pure
function of (seed, iteration, path), so sharding is exact:

  * BDPT  -- rank r renders iterations [r*K, (r+1)*K)  (weak scaling: K per GPU)
  * PT    -- rank r renders its contiguous share of the spp samples

The films are SUMS over iterations/samples, so the only exchange is one
reduce(sum) of the film to rank 0 at the end of a batch (RCCL over xGMI on the
GPU box, gloo in the CPU tests).  Timing = max over ranks; work = sum.
"""


def bdpt_iteration_begin(rank, iters_per_rank):
    """First iteration index of `rank` (iterations of all ranks are disjoint)."""
    if rank < 0 or iters_per_rank < 0:
        raise ValueError("rank and iters_per_rank must be >= 0")
    return rank * iters_per_rank


def pt_sample_range(rank, world, spp):
    """(sample_begin, sample_count) of `rank` when `spp` samples per pixel are
    split across `world` ranks (the first spp % world ranks get one more)."""
    if world <= 0 or not 0 <= rank < world or spp < 0:
        raise ValueError("bad rank/world/spp")
    q, r = divmod(spp, world)
    begin = rank * q + min(rank, r)
    return begin, q + (1 if rank < r else 0)


def _host_backend(dist):
    """gloo reduces host tensors only: device films go through host memory."""
    return dist.get_backend() == "gloo"


def reduce_film(film, dist, dst=0):
    """Sum the ranks' films into rank `dst` (in place there)."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        if _host_backend(dist) and film.device.type != "cpu":
            h = film.cpu()
            dist.reduce(h, dst=dst, op=dist.ReduceOp.SUM)
            if dist.get_rank() == dst:
                film.copy_(h)
        else:
            dist.reduce(film, dst=dst, op=dist.ReduceOp.SUM)
    return film


def job_totals(elapsed_s, rays, dist, device="cpu"):
    """(max elapsed over ranks, total rays of all ranks) -- the bench's
    whole-job numbers."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(elapsed_s), float(rays)
    import torch
    if _host_backend(dist):
        device = "cpu"
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    r = torch.tensor([float(rays)], dtype=torch.float64, device=device)
    dist.all_reduce(r, op=dist.ReduceOp.SUM)
    return float(t.item()), float(r.item())


def min_max(value, dist, device="cpu"):
    """(min, max) of a per-rank float over the ranks (identity for one rank)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value), float(value)
    import torch
    if _host_backend(dist):
        device = "cpu"
    lo = torch.tensor([float(value)], dtype=torch.float64, device=device)
    hi = lo.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    return float(lo.item()), float(hi.item())
