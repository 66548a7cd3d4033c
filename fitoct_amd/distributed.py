"""Chain sharding across GPUs: one process per GPU, one RCCL gather of draws.

SURVEY.md §8e: Stan chains adapt independently, so the chain set partitions
with no data-path collective.  Rank r runs global chains
``[offset_r, offset_r + count_r)``; each chain's random stream is keyed by
(seed, global chain id) (fitoct_config.chain_offset), so the draws of chain c
do not depend on how chains are split across ranks.  Every rank builds the GP
basis from the same inputs (no broadcast).  At the end, one gather moves the
draws to rank 0: with the ``nccl`` backend (RCCL over xGMI on MI355X) the draws
never leave HBM before the gather; with ``gloo`` (CPU tests) they are host
tensors.

This replaces the reference's ``options(mc.cores = detectCores())`` chain
parallelism of rstan (FitOCT.R:13, server.R:469).
"""
from __future__ import annotations

from dataclasses import replace

import numpy as np

from .api import ExpGPProblem, Plan, SampleOutput, SamplerConfig


def shard_range(total: int, world: int, rank: int):
    """Contiguous block partition: (offset, count) of ``rank``'s chains."""
    if not (0 <= rank < world) or total < 0:
        raise ValueError("bad shard request")
    base, rem = divmod(total, world)
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def _gather_rows(t, world, rank, dst=0):
    """Gather equal-shaped tensors to ``dst`` (list on dst, None elsewhere)."""
    import torch
    import torch.distributed as dist
    out = [torch.empty_like(t) for _ in range(world)] if rank == dst else None
    dist.gather(t, gather_list=out, dst=dst)
    return out


def sample_sharded(prob: ExpGPProblem, cfg: SamplerConfig, engine=None, device=None,
                   resume: SampleOutput | None = None):
    """Run ``cfg.chains`` global chains split over the process group; rank 0
    returns the full :class:`SampleOutput` (chains in global order), other ranks
    return their local output without draws.

    ``resume`` (warm restart, :meth:`fitoct_amd.api.Plan.set_init`): a previous run of
    the same global chains -- the full output with every chain, e.g. this function's
    rank-0 output, which the caller must make available on every rank (broadcast it:
    non-zero ranks only get their local block back) -- with the same ``chain_offset``;
    each rank starts its block from that run's last positions, step sizes and inverse
    metrics.  With ``engine`` they reach it as ``engine(prob, cfg, init=(q,
    stepsize, inv_metric))``.

    Without ``engine`` each rank's HIP plan writes its draws into a device tensor;
    with the ``nccl`` backend that tensor is gathered over RCCL directly, with
    ``gloo`` (ranks sharing a GPU in tests and rehearsals) through a host copy.
    ``engine(prob, local_cfg) -> SampleOutput`` replaces the plan by a host-side
    sampler (the CPU tests run the C oracle this way).
    """
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    offset, count = shard_range(cfg.chains, world, rank)
    cmax = -(-cfg.chains // world)
    if count == 0:
        raise ValueError(f"rank {rank} has no chains ({cfg.chains} chains over {world} ranks)")
    local = replace(cfg, chains=count, chain_offset=cfg.chain_offset + offset)
    init = None
    if resume is not None:
        if len(resume.stepsize) != cfg.chains or resume.last_q.shape != (cfg.chains, prob.D):
            raise ValueError("resume must hold the cfg.chains chains of a previous run "
                             "(rank 0's full output, broadcast to every rank)")
        if resume.chain_offset != cfg.chain_offset:
            raise ValueError(f"resume holds global chains from {resume.chain_offset}, this run "
                             f"starts at {cfg.chain_offset}: chains would be paired with others' "
                             "positions")
        blk = slice(offset, offset + count)
        init = (resume.last_q[blk], resume.stepsize[blk], resume.inv_metric[blk])
    nccl = dist.get_backend() == "nccl"
    if engine is None:
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        local = replace(local, device=dev.index)
        with Plan(prob, local) as pl:
            if init is not None:
                pl.set_init(*init)
            info = pl.info
            iters, ncols = info["iters_saved"], info["n_cols"]
            buf = torch.zeros((cmax, iters, ncols), dtype=torch.float64, device=dev)
            pl.run(d_draws=buf.data_ptr(), stream=torch.cuda.current_stream(dev).cuda_stream)
            out = pl.download(with_draws=False)
        if not nccl:          # gloo gathers host tensors
            torch.cuda.current_stream(dev).synchronize()
            buf, dev = buf.cpu(), torch.device("cpu")
    else:
        out = engine(prob, local) if init is None else engine(prob, local, init=init)
        iters, ncols = out.draws.shape[1:]
        buf = torch.zeros((cmax, iters, ncols), dtype=torch.float64)
        buf[:count] = torch.from_numpy(out.draws)
        dev = torch.device("cpu")

    # per-chain scalars ride along in one small tensor: [stepsize, leapfrogs(total), inv_metric, last_q]
    D = out.inv_metric.shape[1]
    meta = np.zeros((cmax, 2 + 2 * D))
    meta[:count, 0] = out.stepsize
    meta[0, 1] = out.total_leapfrogs
    meta[:count, 2:2 + D] = out.inv_metric
    meta[:count, 2 + D:] = out.last_q
    meta_t = torch.from_numpy(meta).to(dev)
    draws_all = _gather_rows(buf, world, rank)
    meta_all = _gather_rows(meta_t, world, rank)
    if rank != 0:
        return out
    counts = [shard_range(cfg.chains, world, r)[1] for r in range(world)]
    draws = torch.cat([d[:n] for d, n in zip(draws_all, counts)]).cpu().numpy()
    meta = torch.cat([m[:n] for m, n in zip(meta_all, counts)]).cpu().numpy()
    total_lf = int(sum(float(m[0, 1]) for m in meta_all))
    return SampleOutput(draws, prob.column_names(), out.warmup_saved, meta[:, 0].copy(),
                        meta[:, 2:2 + D].copy(), meta[:, 2 + D:].copy(), total_lf,
                        out.kernel_ms, out.wall_ms, cfg.chain_offset)


def sample_batch_sharded(probs, cfg: SamplerConfig, engine=None, device=None):
    """FitOCT.R's batch mode over the process group (BASELINE config 5): files are
    split into contiguous blocks over the ranks, each rank samples its block in ONE
    batched launch (:class:`fitoct_amd.api.Batch`), and one gather brings every
    file's draws to rank 0.  File f's chains are global chains
    ``cfg.chain_offset + f*cfg.chains + c`` whatever the split, so the result equals
    a single batch of all files.  Rank 0 returns one :class:`SampleOutput` per file
    (global file order); other ranks return their local outputs.

    Without ``engine`` the batch writes its draws into a device tensor, gathered over
    RCCL with ``nccl`` and through a host copy with ``gloo``; ``engine(prob, cfg) ->
    SampleOutput`` samples one file on the host side instead (CPU tests).
    """
    import torch
    import torch.distributed as dist

    from .api import Batch

    probs = list(probs)
    world, rank = dist.get_world_size(), dist.get_rank()
    F, C = len(probs), cfg.chains
    off, cnt = shard_range(F, world, rank)
    fmax = -(-F // world)
    if cnt == 0:
        raise ValueError(f"rank {rank} has no files ({F} files over {world} ranks)")
    local = replace(cfg, chain_offset=cfg.chain_offset + off * C)
    mine = probs[off:off + cnt]
    nccl = dist.get_backend() == "nccl"
    if engine is None:
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        local = replace(local, device=dev.index)
        with Batch(mine, local) as b:
            iters, ncols = b.info["iters_saved"], b.info["n_cols"]
            buf = torch.zeros((fmax, C, iters, ncols), dtype=torch.float64, device=dev)
            b.run(d_draws=buf.data_ptr(), stream=torch.cuda.current_stream(dev).cuda_stream)
            outs = [b.download(p, with_draws=False) for p in range(cnt)]
        if not nccl:          # gloo gathers host tensors
            torch.cuda.current_stream(dev).synchronize()
            buf, dev = buf.cpu(), torch.device("cpu")
    else:
        outs = [engine(p, replace(local, chain_offset=local.chain_offset + i * C))
                for i, p in enumerate(mine)]
        iters, ncols = outs[0].draws.shape[1:]
        buf = torch.zeros((fmax, C, iters, ncols), dtype=torch.float64)
        for i, o in enumerate(outs):
            buf[i] = torch.from_numpy(o.draws)
        dev = torch.device("cpu")
    D = outs[0].inv_metric.shape[1]
    meta = np.zeros((fmax, C, 2 + 2 * D))
    for i, o in enumerate(outs):
        meta[i, :, 0] = o.stepsize
        meta[i, 0, 1] = o.total_leapfrogs
        meta[i, :, 2:2 + D] = o.inv_metric
        meta[i, :, 2 + D:] = o.last_q
    draws_all = _gather_rows(buf, world, rank)
    meta_all = _gather_rows(torch.from_numpy(meta).to(dev), world, rank)
    if rank != 0:
        return outs
    res = []
    cols = probs[0].column_names()
    for r in range(world):
        o_r, n_r = shard_range(F, world, r)
        d_r, m_r = draws_all[r].cpu().numpy(), meta_all[r].cpu().numpy()
        for i in range(n_r):
            m = m_r[i]
            res.append(SampleOutput(d_r[i].copy(), cols, outs[0].warmup_saved, m[:, 0].copy(),
                                    m[:, 2:2 + D].copy(), m[:, 2 + D:].copy(), int(m[0, 1]),
                                    outs[0].kernel_ms, outs[0].wall_ms,
                                    cfg.chain_offset + (o_r + i) * C))
    return res
