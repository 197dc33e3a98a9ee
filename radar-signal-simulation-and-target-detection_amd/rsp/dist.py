"""Multi-GPU glue: frames are sharded across ranks (one process per GPU); the only
collective is the gather of per-frame detection lists.

Over RCCL (torch.distributed backend "nccl" on ROCm) the gather is an all-gather of
counts followed by a padded all-gather of [n, 5] float64 rows
(frame_idx, Range, Velocity, Angle, Power) -- a few KB per frame, so one xGMI link
is idle-fast.  With the gloo backend the same code runs on CPU tensors (tests).
"""
import numpy as np


def shard_frames(n_frames, rank, world):
    """Contiguous block of frame indices (1-based, as v8:164) owned by ``rank``:
    frames are independent (v8:164-190), so each GPU takes n_frames/world of them."""
    per, extra = divmod(n_frames, world)
    lo = rank * per + min(rank, extra)
    hi = lo + per + (1 if rank < extra else 0)
    return list(range(lo + 1, hi + 1))


def _pack(results):
    rows = []
    for r in results:
        for t in r['final_targets']:
            rows.append((r['frame_idx'], t['Range'], t['Velocity'], t['Angle'], t['Power']))
        if not r['final_targets']:      # keep empty frames visible: one NaN marker row
            rows.append((r['frame_idx'], np.nan, np.nan, np.nan, np.nan))
    return np.asarray(rows, np.float64).reshape(-1, 5)


def gather_targets(results, rank, world, device=None):
    """All-gather every rank's [frame_idx, Range, Velocity, Angle, Power] rows.

    Returns a list of {'frame_idx', 'final_targets'} in (rank, frame) order, identical
    on every rank."""
    counts, bufs = gather_rows(_pack(results), rank, world, device)
    out = []
    for r, (c, b) in enumerate(zip(counts, bufs)):
        frames = {}
        for f, R, V, A, P in b[:c]:
            lst = frames.setdefault(int(f), [])
            if not np.isnan(R):
                lst.append({'Range': R, 'Velocity': V, 'Angle': A, 'Power': P})
        for f in frames:                 # insertion order = the rank's processing order
            out.append({'rank': r, 'frame_idx': f, 'final_targets': frames[f]})
    return out


def gather_rows(rows, rank, world, device=None):
    """The collective itself on packed [n, 5] rows (Plan.results_rows / _pack): all-gather of
    the counts, then a padded all-gather of the rows.  Returns (counts, [per-rank numpy
    arrays of padded rows]), identical on every rank."""
    import torch
    import torch.distributed as dist
    backend = dist.get_backend()
    dev = torch.device('cuda', device) if (backend == 'nccl') else torch.device('cpu')
    local = torch.from_numpy(np.ascontiguousarray(rows, np.float64).reshape(-1, 5)).to(dev)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    m = max(max(counts), 1)
    pad = torch.zeros((m, 5), dtype=torch.float64, device=dev)
    pad[:local.shape[0]] = local
    bufs = [torch.zeros((m, 5), dtype=torch.float64, device=dev) for _ in range(world)]
    dist.all_gather(bufs, pad)
    return counts, [b.cpu().numpy() for b in bufs]
