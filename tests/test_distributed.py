"""Chain sharding over a process group (gloo, world_size 2): the gathered draws on
rank 0 equal a single-process run of all chains, for even and uneven splits.

CPU: the engine on each rank is the C oracle.  GPU (``-m gpu``): both ranks run the
HIP plan on cuda:0 into device buffers -- the code path the nccl backend takes on a
node, with the one collective done through a host copy because RCCL refuses two
ranks on one device -- and the gathered draws equal a single plan bit for bit."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from fitoct_amd.distributed import shard_range


def test_shard_range_partitions():
    for total in [1, 7, 8, 1024, 8192, 1001]:
        for world in [1, 2, 3, 8]:
            if total < world:
                continue
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0
            for (o1, c1), (o2, _) in zip(spans, spans[1:]):
                assert o1 + c1 == o2
            assert sum(c for _, c in spans) == total
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _problem():
    from fitoct_amd import ExpGPProblem
    from fitoct_amd.synth import default_prior, synth_decay
    t0, S0 = default_prior()
    d = synth_decay(40, "sincExp2", 9)
    return ExpGPProblem(d["x"], d["y"], d["uy"], Nn=4, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type="lasso")


def _oracle_engine(prob, cfg, init=None):
    from fitoct_amd.api import SampleOutput
    from oracle import nuts_c
    kw = {} if init is None else dict(q_init=init[0], init_stepsize=init[1],
                                      init_inv_metric=init[2])
    o = nuts_c.sample(prob, cfg, nthreads=1, **kw)
    return SampleOutput(o["draws"], prob.column_names(), cfg.warmup, o["stepsize"],
                        o["inv_metric"], np.zeros_like(o["inv_metric"]),
                        int(o["leapfrogs"].sum()), 0.0, 0.0, cfg.chain_offset)


def _worker(rank, world, port, chains, outdir):
    import torch.distributed as dist
    from fitoct_amd.api import SamplerConfig
    from fitoct_amd.distributed import sample_sharded
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        cfg = SamplerConfig(chains=chains, warmup=30, samples=20, seed=21, max_treedepth=5)
        out = sample_sharded(_problem(), cfg, engine=_oracle_engine)
        if rank == 0:
            np.savez(os.path.join(outdir, "gathered.npz"), draws=out.draws,
                     stepsize=out.stepsize, lf=out.total_leapfrogs)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("chains", [4, 5])
def test_gloo_world2_gather_equals_single_run(tmp_path, chains):
    from fitoct_amd.api import SamplerConfig
    mp.spawn(_worker, args=(2, _free_port(), chains, str(tmp_path)), nprocs=2, join=True)
    got = np.load(tmp_path / "gathered.npz")
    ref = _oracle_engine(_problem(), SamplerConfig(chains=chains, warmup=30, samples=20,
                                                   seed=21, max_treedepth=5))
    np.testing.assert_array_equal(got["draws"], ref.draws)
    np.testing.assert_array_equal(got["stepsize"], ref.stepsize)
    assert int(got["lf"]) == ref.total_leapfrogs


def _batch_problems():
    from fitoct_amd import ExpGPProblem
    from fitoct_amd.synth import MODULATIONS, default_prior, synth_decay
    t0, S0 = default_prior()
    out = []
    for f in range(5):
        d = synth_decay(30 + 3 * f, MODULATIONS[f % 4], 100 + f)
        out.append(ExpGPProblem(d["x"], d["y"], d["uy"], Nn=4, gridType="extremal", theta0=t0,
                                Sigma0=S0, prior_type="normal"))
    return out


def _batch_worker(rank, world, port, outdir):
    import torch.distributed as dist
    from fitoct_amd.api import SamplerConfig
    from fitoct_amd.distributed import sample_batch_sharded
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        cfg = SamplerConfig(chains=2, warmup=20, samples=10, seed=5, max_treedepth=4)
        outs = sample_batch_sharded(_batch_problems(), cfg, engine=_oracle_engine)
        if rank == 0:
            np.savez(os.path.join(outdir, "batch.npz"),
                     draws=np.stack([o.draws for o in outs]),
                     offsets=np.array([o.chain_offset for o in outs]))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_batch_files_equal_single_runs(tmp_path):
    """Config 5 over ranks: 5 files split 3 + 2; file f's chains are global chains
    f*chains + c, so each file equals its own single run at that chain offset."""
    from fitoct_amd.api import SamplerConfig
    mp.spawn(_batch_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    got = np.load(tmp_path / "batch.npz")
    np.testing.assert_array_equal(got["offsets"], [0, 2, 4, 6, 8])
    for f, prob in enumerate(_batch_problems()):
        ref = _oracle_engine(prob, SamplerConfig(chains=2, warmup=20, samples=10, seed=5,
                                                 max_treedepth=4, chain_offset=2 * f))
        np.testing.assert_array_equal(got["draws"][f], ref.draws)


def _hip_worker(rank, world, port, chains, outdir, batch):
    import torch
    import torch.distributed as dist
    from fitoct_amd.api import SamplerConfig
    from fitoct_amd.distributed import sample_batch_sharded, sample_sharded
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        if batch:
            cfg = SamplerConfig(chains=2, warmup=20, samples=10, seed=5, max_treedepth=5)
            outs = sample_batch_sharded(_batch_problems(), cfg)
            if rank == 0:
                np.savez(os.path.join(outdir, "gathered.npz"),
                         draws=np.stack([o.draws for o in outs]))
        else:
            cfg = SamplerConfig(chains=chains, warmup=60, samples=40, seed=21, max_treedepth=6)
            out = sample_sharded(_gpu_problem(), cfg)
            if rank == 0:
                np.savez(os.path.join(outdir, "gathered.npz"), draws=out.draws,
                         stepsize=out.stepsize, lf=out.total_leapfrogs)
    finally:
        dist.destroy_process_group()


def _gpu_problem():
    from fitoct_amd import ExpGPProblem
    from fitoct_amd.synth import default_prior, synth_decay
    t0, S0 = default_prior()
    d = synth_decay(512, "sincExp2", 9)
    return ExpGPProblem(d["x"], d["y"], d["uy"], Nn=10, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type="horseshoe")


@pytest.mark.gpu
@pytest.mark.parametrize("chains", [64, 37])
def test_hip_plan_sharded_gather_equals_single_plan(tmp_path, chains):
    from fitoct_amd.api import SamplerConfig, sample
    mp.spawn(_hip_worker, args=(2, _free_port(), chains, str(tmp_path), False), nprocs=2,
             join=True)
    got = np.load(tmp_path / "gathered.npz")
    ref = sample(_gpu_problem(), SamplerConfig(chains=chains, warmup=60, samples=40, seed=21,
                                               max_treedepth=6))
    np.testing.assert_array_equal(got["draws"], ref.draws)
    np.testing.assert_array_equal(got["stepsize"], ref.stepsize)
    assert int(got["lf"]) == ref.total_leapfrogs


@pytest.mark.gpu
def test_hip_batch_sharded_gather_equals_single_batch(tmp_path):
    from fitoct_amd.api import SamplerConfig, sample_batch
    mp.spawn(_hip_worker, args=(2, _free_port(), 0, str(tmp_path), True), nprocs=2, join=True)
    got = np.load(tmp_path / "gathered.npz")["draws"]
    ref = sample_batch(_batch_problems(), SamplerConfig(chains=2, warmup=20, samples=10, seed=5,
                                                        max_treedepth=5))
    np.testing.assert_array_equal(got, np.stack([o.draws for o in ref]))


def _resume_state(chains):
    """A previous run's end state for every global chain (oracle run, last draw mapped
    back to the unconstrained space)."""
    from fitoct_amd.api import SampleOutput, SamplerConfig
    prob = _problem()
    o = _oracle_engine(prob, SamplerConfig(chains=chains, warmup=40, samples=10, seed=3,
                                           max_treedepth=5))
    last = o.draws[:, -1, 7:7 + prob.D]
    logc = np.array([k < 3 or k >= 3 + prob.Nn for k in range(prob.D)])
    q = last.copy()
    q[:, logc] = np.log(last[:, logc])
    return SampleOutput(None, [], 0, o.stepsize, o.inv_metric, q, 0, 0.0, 0.0)


def _resume_worker(rank, world, port, chains, outdir):
    import torch.distributed as dist
    from fitoct_amd.api import SamplerConfig
    from fitoct_amd.distributed import sample_sharded
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        cfg = SamplerConfig(chains=chains, warmup=0, samples=20, seed=22, max_treedepth=5,
                            adapt_engaged=False)
        out = sample_sharded(_problem(), cfg, engine=_oracle_engine,
                             resume=_resume_state(chains))
        if rank == 0:
            np.savez(os.path.join(outdir, "resumed.npz"), draws=out.draws, stepsize=out.stepsize)
    finally:
        dist.destroy_process_group()


def test_gloo_world2_resume_equals_single_run(tmp_path):
    """Warm restart over the process group: each rank starts its chain block from the
    previous run's end state, and the gathered draws equal one process resuming all
    chains (uneven split: 5 chains over 2 ranks)."""
    from fitoct_amd.api import SamplerConfig
    chains = 5
    mp.spawn(_resume_worker, args=(2, _free_port(), chains, str(tmp_path)), nprocs=2,
             join=True)
    got = np.load(tmp_path / "resumed.npz")
    st = _resume_state(chains)
    ref = _oracle_engine(_problem(), SamplerConfig(chains=chains, warmup=0, samples=20, seed=22,
                                                   max_treedepth=5, adapt_engaged=False),
                         init=(st.last_q, st.stepsize, st.inv_metric))
    np.testing.assert_array_equal(got["draws"], ref.draws)
    np.testing.assert_array_equal(got["stepsize"], st.stepsize)


def _hip_resume_worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist
    from fitoct_amd.api import SamplerConfig, sample
    from fitoct_amd.distributed import sample_sharded
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        prev = sample(_gpu_problem(), SamplerConfig(chains=37, warmup=60, samples=10, seed=21,
                                                    max_treedepth=6))
        cfg = SamplerConfig(chains=37, warmup=0, samples=30, seed=23, max_treedepth=6,
                            adapt_engaged=False)
        out = sample_sharded(_gpu_problem(), cfg, resume=prev)
        if rank == 0:
            np.savez(os.path.join(outdir, "resumed.npz"), draws=out.draws)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_hip_plan_sharded_resume_equals_single_plan(tmp_path):
    """Warm restart through the HIP plans of two ranks (37 chains: 19 + 18) equals one
    plan resuming all chains, bit for bit."""
    from fitoct_amd.api import SamplerConfig, sample
    mp.spawn(_hip_resume_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    got = np.load(tmp_path / "resumed.npz")["draws"]
    prev = sample(_gpu_problem(), SamplerConfig(chains=37, warmup=60, samples=10, seed=21,
                                                max_treedepth=6))
    ref = sample(_gpu_problem(), SamplerConfig(chains=37, warmup=0, samples=30, seed=23,
                                               max_treedepth=6, adapt_engaged=False), resume=prev)
    np.testing.assert_array_equal(got, ref.draws)
