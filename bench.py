"""Headline benchmark: posterior draws/sec of FitOCT's ExpGP posterior on MI355X.

Workload (BASELINE.json configs[2]): ``fitExpGP`` + horseshoe prior
(Tests/horseShoePrior.stan, nu = 1), N = 2048 depth bins, Nn = 15 extremal control
points (ctrlParams.yaml:3-5), 1024 chains per GPU, 500 warmup + 1000 sampling
iterations per chain (FitOCT.R:43-44), adapt_delta 0.8, max_treedepth 10, all
draws (warmup included, save_warmup) written to HBM.  Synthetic data: the
restated synthData.R decay (fitoct_amd/synth.py, 'sincExp').

A *step* = one complete sampler run of the local chains (plan launch: init,
step-size search, adaptation, sampling); for N > 1 ranks it also includes the
single RCCL gather of every rank's draws to rank 0.  Inputs are staged in HBM
(plan creation) before the timed region.  Each step uses a fresh seed.

    value = n_gpus * chains * samples / (max over ranks of wall per step)

Extra objects on the JSON line: ``roofline`` (FP64 vector roofline of the
sampler kernel: algorithmic flop F_grad = 4*N*Nn + 20*N per gradient, SURVEY.md
§8d, x leapfrogs counted by the kernel / kernel time from HIP events on the
launch stream; HBM traffic from the committed rocprofv3 PMC summary) and
``cpu_baseline`` (the C oracle NUTS on this host's cores, bounded sample, scaled
to the same unit -- see DESIGN.md §Measurement).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_BINS, NN, CHAINS, WARMUP_IT, SAMPLES = 2048, 15, 1024, 500, 1000
# BASELINE.json configs that run on the sampler (--config K = configs[K-1]).  The
# headline line is config 3; 2 and 4 are secondary measurements (config 4's
# 8192 chains are 1024 per GPU over 8 GPUs: weak scaling of the same per-GPU shape).
CONFIGS = {
    2: dict(prior="normal", N=512, chains=128),
    3: dict(prior="horseshoe", N=2048, chains=1024),
    4: dict(prior="lasso", N=4096, chains=1024),
    # FitOCT.R batch mode: 256 synthetic files (the 4 modulations of synthData.R:21,35,49,
    # 63 at N=481), 4 chains each, ctrlParams.yaml's 100 warmup + 100 draws, Nn=15
    # extremal, normal prior; files sharded in contiguous blocks over the ranks (strong scaling)
    5: dict(prior="normal", N=481, chains=4, files=256, iters=(100, 100)),
}
# the hard-geometry sub-line's step seed: fixed, whatever --steps is, so its R-hat never
# depends on which seed a step count selects (tests/test_gpu_sampler.py runs it and 1001, 1019)
HARD_SEED = 1000
FP64_VALU_PEAK_TF = 78.6          # MI355X FP64 vector peak (vendor spec; 1/2 of FP32 vector)
HBM_PEAK_GBS = 8000.0
# PMC traffic summaries (scripts/pmc_traffic.sh [config]), newest round first, matched to
# a bench line by its workload string
TRAFFIC_GLOB = os.path.join(ROOT, "profiles", "r*_pmc_traffic*.json")


def f_grad(N, Nn):
    return 4 * N * Nn + 20 * N     # SURVEY.md §8d algorithmic flop per gradient


def make_problem(prior="horseshoe", N=N_BINS):
    from fitoct_amd import ExpGPProblem
    from fitoct_amd.synth import default_prior, synth_decay
    t0, S0 = default_prior()
    d = synth_decay(N, "sincExp", 1234)
    # lasso lambda_s = 10 mirrors Tests/testGamma.R:35
    return ExpGPProblem(d["x"], d["y"], d["uy"], dataType=2, Nn=NN, gridType="extremal",
                        theta0=t0, Sigma0=S0, prior_type=prior, nu=1.0, lambda_scale=10.0)


def make_config(seed, chains, offset, device, warmup_it, samples, adapt_delta=0.8,
                max_treedepth=10):
    from fitoct_amd import SamplerConfig
    return SamplerConfig(chains=chains, chain_offset=offset, warmup=warmup_it, samples=samples,
                         seed=seed, adapt_delta=adapt_delta, max_treedepth=max_treedepth,
                         device=device)


def host_cpu_info():
    """The host's CPUs as the bench sees them: the node's logical CPUs (``nproc``
    of the whole machine), the CPUs this process may run on (affinity), the
    cgroup CPU quota (``cpu.max``; a shared GPU box grants each job a share of the
    node), and the ``lscpu`` model name."""
    node = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = node
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    sockets = set()
    cores = {}   # logical CPU -> (socket, core): SMT siblings share a physical core
    try:
        with open("/proc/cpuinfo") as f:
            cpu = sock = None
            for ln in f:
                k, _, v = ln.partition(":")
                k, v = k.strip(), v.strip()
                if k == "processor":
                    cpu = int(v)
                elif k == "physical id":
                    sock = v
                    sockets.add(v)
                elif k == "core id" and cpu is not None:
                    cores[cpu] = (sock, v)
    except (OSError, ValueError):
        pass
    share = min(avail, quota) if quota else avail
    try:
        aff = sorted(os.sched_getaffinity(0))
    except AttributeError:
        aff = list(range(node))
    node_phys = len(set(cores.values())) or None
    aff_phys = len({cores[c] for c in aff if c in cores}) or None
    return {"node_cpus": node, "affinity_cpus": avail, "cgroup_quota_cpus": quota,
            "share_cpus": share, "sockets": len(sockets) or None, "model": model,
            # SMT: the node's physical cores and the physical cores the affinity mask spans
            # (a quota of share_cpus logical CPUs may run on fewer cores than CPUs)
            "node_physical_cores": node_phys, "affinity_physical_cores": aff_phys,
            "smt_threads_per_core": (round(node / node_phys, 2) if node_phys else None)}


def cpu_baseline(prob, gpu_lf_per_step, draws_per_step, adapt_delta=0.8, max_treedepth=10,
                 same_length=None):
    """C oracle (oracle/fitoct_oracle.c, OpenMP over chains): a bounded run of the
    same problem, one chain per host thread (250 warmup + 250 draws, ~10-20 s), its
    leapfrog rate scaled by the GPU step's leapfrogs per draw.  It runs on every CPU
    this job may use (affinity and cgroup quota: the job's share of a shared node);
    chains are independent, so the node-wide rate is also given as the measured
    per-thread rate times the node's logical CPUs (``value_node_est``).

    ``same_length`` = (W, S): also a direct run at the workload's own per-chain length --
    one chain per thread of the share, W warmup + S draws each, value = chains x S / wall,
    no scaling (``value_measured_same_length``)."""
    from oracle import nuts_c
    hw = host_cpu_info()
    threads = hw["share_cpus"]
    W, S = 250, 250
    cfg = make_config(7, threads, 900_000, 0, W, S, adapt_delta, max_treedepth)
    t = time.perf_counter()
    o = nuts_c.sample(prob, cfg, nthreads=threads)
    wall = time.perf_counter() - t
    lf = int(o["leapfrogs"].sum())
    lf_rate = lf / wall
    value = draws_per_step * lf_rate / gpu_lf_per_step
    post = o["draws"][:, W:, :] if cfg.save_warmup else o["draws"]
    direct = {}
    if same_length is not None:
        W2, S2 = same_length
        cfg2 = make_config(8, threads, 950_000, 0, W2, S2, adapt_delta, max_treedepth)
        t2 = time.perf_counter()
        o2 = nuts_c.sample(prob, cfg2, nthreads=threads)
        wall2 = time.perf_counter() - t2
        v2 = threads * S2 / wall2
        lf2 = float(o2["leapfrogs"].sum())
        direct = {"value_measured_same_length": round(v2, 2),
                  "same_length_sample": (f"C oracle NUTS, {threads} chains x ({W2} warmup + {S2} "
                                         f"draws) on {threads} threads, {wall2:.1f} s: chains x "
                                         f"draws / wall, no scaling"),
                  "measured_over_scaled": round(v2 / value, 3),
                  # the ratio's two factors: the gradient rate of the longer run over the
                  # sample's (the same problem on the same threads: ~1) and the GPU step's
                  # gradients per draw over this run's own (its 16 chains' tree depths)
                  "same_length_grad_rate_ratio": round(lf2 / wall2 / lf_rate, 3),
                  "same_length_grads_per_draw_ratio": round(
                      (gpu_lf_per_step / draws_per_step) / (lf2 / (threads * S2)), 3)}
    return {"means": np.nanmean(post, axis=(0, 1)), "lf_rate": lf_rate, "value": value,
            **direct,
            "unit": "draws/s",
            "cores": threads, "kind": "port",
            "value_node_est": value * hw["node_cpus"] / threads,
            "host": hw,
            "sample": (f"C oracle NUTS, {threads} chains x ({W} warmup + {S} draws) of the same "
                       f"problem on {threads} threads (this job's CPU share of a "
                       f"{hw['node_cpus']}-CPU node, {hw['model'] or 'unknown model'}): {lf} "
                       f"gradients in {wall:.1f} s ({lf_rate:.3g} grad/s); scaled by the GPU "
                       f"step's {gpu_lf_per_step / draws_per_step:.1f} gradients per "
                       f"post-warmup draw; value_node_est = value x {hw['node_cpus']}/{threads}"),
            "wall_s": round(wall, 2)}


def convergence(draws, W_saved, cols):
    """Split and rank-normalised R-hat of the post-warmup draws over the parameter
    columns (theta, z / yGP, the scales, sigma, br; the horseshoe's inverse-gamma
    auxiliaries r2_* excluded), with and without the funnel-trapped chains, and the three
    worst columns by name.  Trapped: ``fitoct_amd.stanfit.trapped_chains``, the fixed rule
    (more than half of a chain's transitions diverge over the run or over either half of
    it); ``stuck_chains_whole_run`` counts by rounds 1-3's whole-run rule."""
    from fitoct_amd.stanfit import rank_rhat, split_rhat_ess, trapped_chains, trapped_whole_run
    post = draws[:, W_saved:, :]
    par = [j for j, n in enumerate(cols) if j >= 7 and not n.startswith("r2_")]
    rhe = {cols[j]: split_rhat_ess(post[:, :, j]) for j in par}
    rh = {k: v[0] for k, v in rhe.items()}
    ess = {k: v[1] for k, v in rhe.items()}   # rstan n_eff over all chains
    rrh = {cols[j]: rank_rhat(post[:, :, j]) for j in par}   # Vehtari et al. 2021
    stuck = trapped_chains(post[:, :, 5])
    free = post[~stuck]
    rh_free = {cols[j]: split_rhat_ess(free[:, :, j])[0] for j in par} if stuck.any() else rh
    rrh_free = {cols[j]: rank_rhat(free[:, :, j]) for j in par} if stuck.any() else rrh

    def worst(d):
        return [[k, round(float(v), 5)] for k, v in sorted(d.items(), key=lambda t: -t[1])[:3]]
    return {"rhat_max": round(max(rh.values()), 5), "stuck_chains": int(stuck.sum()),
            "stuck_chains_whole_run": int(trapped_whole_run(post[:, :, 5]).sum()),
            "rhat_max_excl_stuck": round(max(rh_free.values()), 5),
            "rank_rhat_max": round(max(rrh.values()), 5),
            "rank_rhat_max_excl_stuck": round(max(rrh_free.values()), 5),
            "divergent_frac": round(float(post[:, :, 5].mean()), 5),
            "rhat_worst_columns": worst(rh), "rank_rhat_worst_columns": worst(rrh),
            # slow mixing vs trapping: with nothing trapped, split R-hat - 1 ~ 1 / (bulk ESS
            # per chain), e.g. config 4's yGP.6-8 (~90 per 1000 draws)
            "ess_per_chain_min": round(min(ess.values()) / post.shape[0], 1),
            "ess_per_chain_lowest_columns": [[k, round(v / post.shape[0], 1)] for k, v in
                                             sorted(ess.items(), key=lambda t: t[1])[:3]]}


def load_traffic(workload):
    import glob
    for path in sorted(glob.glob(TRAFFIC_GLOB), reverse=True):
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        if t.get("workload") == workload:
            t["source"] = os.path.relpath(path, ROOT)
            return t
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS),
                    help="BASELINE.json configs[K-1]; 3 is the headline")
    ap.add_argument("--chains", type=int, default=0, help="chains per GPU (0: the config's)")
    ap.add_argument("--iters", type=str, default=f"{WARMUP_IT},{SAMPLES}",
                    help="sampler warmup,samples per chain")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--precision", default="f64", choices=["f64", "mixed"])
    ap.add_argument("--adapt-delta", type=float, default=0.8,
                    help="0.8: rstan's default (the headline); 0.99 with --max-treedepth 12 is "
                         "the reference's hard-geometry profile (Tests/testGamma.R:45)")
    ap.add_argument("--max-treedepth", type=int, default=10)
    ap.add_argument("--no-hard", action="store_true",
                    help="skip the hard-geometry sub-line (one extra config-3 step at "
                         "adapt_delta 0.99, max_treedepth 12; N = 1 only)")
    ap.add_argument("--devices", type=int, default=0,
                    help="the single-process route: one plan over the C ABI's device list "
                         "(fitoct_config.devices, what R's fitExpGP(n_gpus = N) drives through "
                         ".Call; FitOCT.R:110, server.R:408) on N GPUs, the config's chains per "
                         "GPU, the in-process xGMI gather into one device buffer inside the "
                         "step; run without torchrun (--gpus 1).  0 / 1: one device")
    ap.add_argument("--device-ids", type=str, default="",
                    help="explicit ordinals for --devices, e.g. 0,0 rehearses two entries on "
                         "one GPU")
    ap.add_argument("--no-device-list", action="store_true",
                    help="under torchrun (N > 1): skip the device-list sub-line that rank 0 "
                         "times over all N GPUs after the per-rank steps")
    args = ap.parse_args()
    if args.config == 5 and args.iters == f"{WARMUP_IT},{SAMPLES}":
        args.iters = "%d,%d" % CONFIGS[5]["iters"]
    W_it, S_it = (int(v) for v in args.iters.split(","))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    dist = None
    # FITOCT_BENCH_BACKEND=gloo rehearses the multi-rank path with ranks sharing
    # GPUs (RCCL refuses two ranks on one device); the driver's runs use nccl.
    backend = os.environ.get("FITOCT_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)
    dev_list = ()
    if args.devices > 1 or args.device_ids:
        if world > 1:
            raise SystemExit("--devices is the single-process route: run it without torchrun")
        dev_list = (tuple(int(v) for v in args.device_ids.split(",")) if args.device_ids
                    else tuple(range(args.devices)))
        if args.devices > 1 and len(dev_list) != args.devices:
            raise SystemExit(f"--devices {args.devices} but --device-ids lists {len(dev_list)}")
        if max(dev_list) >= ndev:
            raise SystemExit(f"--devices: device {max(dev_list)} of {ndev} visible")

    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    cdev = dev if backend == "nccl" else torch.device("cpu")   # where collectives run

    if args.config == 5:
        return bench_batch(args, world, rank, local, dev, dist, backend, cdev, W_it, S_it,
                           dev_list)

    from fitoct_amd import Plan
    from fitoct_amd.api import SamplerConfig  # noqa: F401  (import check)

    conf = CONFIGS[args.config]
    N_bins = conf["N"]
    prob = make_problem(conf["prior"], N_bins)
    C = args.chains or conf["chains"]
    offset = rank * C
    n_units = len(dev_list) or world      # GPUs the job's chains span (ranks or list entries)
    C_plan = C * max(1, len(dev_list))    # chains of this process's plan

    def plan_for(step):
        cfg = make_config(1000 + step, C_plan, offset, local, W_it, S_it, args.adapt_delta,
                          args.max_treedepth)
        cfg.precision = args.precision
        cfg.devices = dev_list
        return Plan(prob, cfg)

    stream = torch.cuda.current_stream(dev)
    info = None
    bufs = {}

    def run_step(pl):
        nonlocal info
        info = pl.info
        key = info["draws_bytes"]
        if key not in bufs:
            bufs[key] = torch.empty(key // 8, dtype=torch.float64, device=dev)
            if world > 1 and rank == 0:
                bufs["gather"] = [torch.empty(key // 8, dtype=torch.float64, device=cdev)
                                  for _ in range(world)]
        buf = bufs[key]
        # a device list runs each GPU on a private stream of the library (stream = NULL),
        # and gathers every block into `buf` (on this process's device) before returning
        pl.run(d_draws=buf.data_ptr(), stream=0 if dev_list else stream.cuda_stream)
        if world > 1:   # one gather of every rank's draws to rank 0 (RCCL over xGMI)
            src = buf if backend == "nccl" else buf.cpu()
            dist.gather(src, gather_list=bufs.get("gather") if rank == 0 else None, dst=0)
        return buf

    # ---- untimed warmup steps -------------------------------------------------
    for w in range(args.warmup):
        with plan_for(-1 - w) as pl:
            run_step(pl)
        if rank == 0:   # progress on stderr (a long run stays visibly alive; stdout is the line)
            print(f"[bench] warmup step {w + 1}/{args.warmup} done", file=sys.stderr, flush=True)
    torch.cuda.synchronize()

    plans = [plan_for(s) for s in range(args.steps)]     # inputs staged in HBM up front
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_ms = []
    for i, pl in enumerate(plans):
        run_step(pl)
        kernel_ms.append(pl.download(with_draws=False).kernel_ms)
        if rank == 0:
            print(f"[bench] step {i + 1}/{args.steps}: kernel {kernel_ms[-1]:.1f} ms",
                  file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([wall], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())

    outs = [pl.download(with_draws=(i == len(plans) - 1)) for i, pl in enumerate(plans)]
    lf_steps = [o.total_leapfrogs for o in outs]
    if dist is not None:
        t = torch.tensor(lf_steps, dtype=torch.float64, device=cdev)
        dist.all_reduce(t)
        lf_all = t.cpu().numpy()
    else:
        lf_all = np.array(lf_steps, dtype=np.float64)

    ms_per_step = wall * 1e3 / args.steps
    draws_step = world * C_plan * S_it
    value = draws_step / (ms_per_step / 1e3)

    # convergence of the last step: split R-hat over parameters, over every rank's chains (the
    # gathered draws: rank 0 holds the whole job's last step after its gather)
    last = outs[-1].draws
    cols = prob.column_names()
    W_saved = outs[-1].warmup_saved
    conv_draws = last
    if world > 1 and rank == 0 and "gather" in bufs:
        shp = last.shape
        conv_draws = np.concatenate([g.cpu().numpy().reshape(shp) for g in bufs["gather"]])
    conv = convergence(conv_draws, W_saved, cols)
    conv["rhat_chains"] = int(conv_draws.shape[0])
    lf_per_draw = float(np.mean(lf_steps)) / (C_plan * (W_it + S_it))

    workload = (f"fitExpGP+{conf['prior']} N={N_bins} Nn={NN} {C} chains/GPU "
                f"W={W_it} S={S_it} treedepth<={args.max_treedepth}"
                + ("" if args.adapt_delta == 0.8 else f" adapt_delta={args.adapt_delta:g}"))
    kms = float(np.mean(kernel_ms))
    flops = f_grad(N_bins, NN) * float(np.mean(lf_steps))
    achieved = flops / (kms / 1e3) / 1e12
    traffic = load_traffic(workload)
    roof = {"bound": "valu", "achieved": round(achieved, 3), "peak": FP64_VALU_PEAK_TF,
            "unit": "TFLOP/s", "frac": round(achieved / FP64_VALU_PEAK_TF, 4),
            "traffic": traffic["bytes_per_launch"] if traffic else None,
            "kernel": "nuts_kernel", "kernel_ms": round(kms, 2),
            "flop_per_gradient": f_grad(N_bins, NN),
            "gradients_per_launch": int(np.mean(lf_steps))}
    if traffic:
        roof["hbm_gbs"] = round(traffic["bytes_per_launch"] / (kms / 1e3) / 1e9, 2)
        roof["hbm_frac"] = round(roof["hbm_gbs"] / HBM_PEAK_GBS, 5)
        roof["traffic_source"] = traffic["source"]

    line = {
        "metric": ("posterior draws/sec (all chains), ExpGP N=2048 @ 1024 chains; R-hat"
                   if args.config == 3 else f"posterior draws/sec (all chains), config {args.config}"),
        "value": round(value, 2), "unit": "draws/s", "n_gpus": n_units, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64" if args.precision == "f64"
        else "f32-sweep/f64-state", "data": "synthetic (restated synthData.R sincExp decay)",
        "config": {"workload": workload, "prior": conf["prior"], "N": N_bins, "Nn": NN,
                   "chains_per_gpu": C, "global_chains": n_units * C, "warmup_iters": W_it,
                   "samples": S_it, "adapt_delta": args.adapt_delta,
                   "max_treedepth": args.max_treedepth,
                   "parallelism": (f"chains sharded over {world} GPU(s)" if not dev_list else
                                   f"device list {list(dev_list)} in one process "
                                   "(fitoct_config.devices: R fitExpGP(n_gpus) route)"),
                   "route": ("device-list" if dev_list else
                             "torch.distributed" if world > 1 else "single-device")},
        **conv,
        "gradients_per_iteration": round(lf_per_draw, 1),
        # sampling phase alone: the kernel is gradient-bound, so its time is
        # apportioned by the post-warmup share of the last step's gradients (rank 0's chains)
        "sampling_only_draws_per_s_est": round(
            draws_step / (kms / 1e3 * float(last[:, W_saved:, 4].sum()) / outs[-1].total_leapfrogs), 1),
        "total_gradients_per_step": float(lf_all.mean()),
        "roofline": roof,
    }
    if rank == 0 and n_units == 1 and not args.no_cpu:
        cb = cpu_baseline(prob, float(np.mean(lf_steps)), C * S_it, args.adapt_delta,
                          args.max_treedepth, same_length=(W_it, S_it))
        o_means = cb.pop("means")
        line["cpu_baseline"] = cb
        # north star: posterior means within 1 % of the CPU path on the same inputs.
        # GPU: this step's chains after warmup; oracle: the bounded CPU sample above
        # (its own Monte-Carlo error, ~0.1 % on theta, is part of the figure).
        g_means = np.nanmean(last[:, W_saved:, :], axis=(0, 1))
        rel = {n: round(float(abs(g_means[j] - o_means[j]) / abs(o_means[j])), 6)
               for j, n in enumerate(cols) if n.startswith("theta") or n in ("sigma", "br")}
        line["posterior_mean_relerr_vs_cpu"] = rel
    for pl in plans:
        pl.close()
    bufs.clear()
    if (args.config == 3 and n_units == 1 and not args.no_hard and args.adapt_delta == 0.8
            and args.chains == 0 and (W_it, S_it) == (WARMUP_IT, SAMPLES)):
        line["hard_geometry"] = hard_geometry(prob, C, local, dev, W_it, S_it, cols,
                                              line.get("cpu_baseline"),
                                              o_means if "cpu_baseline" in line else None,
                                              seed=HARD_SEED)
    if world > 1 and not args.no_device_list:
        # the route R takes (.Call -> fitoct_config.devices), timed on the same node: rank 0
        # alone drives every GPU of the job from one process while the other ranks wait on
        # a host (gloo) barrier, so no collective kernel occupies their GPUs meanwhile
        hb = dist.new_group(backend="gloo")
        dist.barrier(group=hb)
        if rank == 0:
            try:   # a side measurement: it must not cost the headline line
                line["device_list"] = device_list_leg(
                    lambda step, devs: Plan(prob, _dl_config(args, C * len(devs), W_it, S_it,
                                                             step, devs)),
                    _dl_devices(world, ndev), C * S_it, dev, f_grad(N_bins, NN))
            except Exception as e:   # noqa: BLE001
                line["device_list"] = {"error": f"{type(e).__name__}: {e}"}
        dist.barrier(group=hb)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def _dl_devices(world, visible):
    """GPUs of the device-list sub-line: the job's, one entry per rank (one node, one rank
    per GPU), each a VISIBLE ordinal: rank r -> r mod visible, so ranks sharing fewer GPUs
    (a rehearsal on one GPU: 0,0,...) list each card once per rank that uses it.
    FITOCT_BENCH_DEVICE_LIST=0,1,... overrides; an ordinal outside [0, visible) fails here,
    before the leg's timed region, with a message."""
    env = os.environ.get("FITOCT_BENCH_DEVICE_LIST", "")
    devs = tuple(int(v) for v in env.split(",") if v) or tuple(r % max(visible, 1)
                                                               for r in range(world))
    bad = [d for d in devs if not 0 <= d < visible]
    if bad:
        raise ValueError(f"device list {list(devs)}: ordinals {bad} are not among the "
                         f"{visible} visible GPU(s)")
    return devs


def _dl_config(args, chains, W_it, S_it, step, devs):
    cfg = make_config(1000 + step, chains, 0, devs[0], W_it, S_it, args.adapt_delta,
                      args.max_treedepth)
    cfg.devices = devs
    return cfg


def device_list_leg(make, devs, draws_per_gpu, dev, flop_per_grad, is_batch=False):
    """One step of the single-process route over `devs` (the C ABI's device list:
    one host thread per GPU inside libfitoct, blocks gathered over xGMI into one
    buffer on `dev` before the call returns), timed like a headline step: the
    plan (basis, staging) is created before the timer.  `make(step, devs)` builds
    the plan or batch (seed 1000 + step, the first timed step's seed)."""
    import torch
    with make(0, devs) as pl:
        buf = torch.empty(pl.info["draws_bytes"] // 8, dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pl.run(d_draws=buf.data_ptr())
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        o = pl.download(0, with_draws=False) if is_batch else pl.download(with_draws=False)
        kms, lf = o.kernel_ms, (None if is_batch else o.total_leapfrogs)
    res = {"route": "fitoct_config.devices (one process, one host thread per GPU; "
                    "R fitExpGP(n_gpus) via .Call)",
           "devices": list(devs), "value": round(len(devs) * draws_per_gpu / wall, 2),
           "unit": "draws/s", "ms_per_step": round(wall * 1e3, 2),
           "kernel_ms_max_over_devices": round(kms, 2), "steps": 1,
           "gather": "in-process hipMemcpyPeer of every block into one buffer on GPU "
                     f"{dev.index}, inside the step"}
    if lf:
        res["gradients_per_launch"] = lf
        res["roofline_frac_per_gpu"] = round(flop_per_grad * lf / len(devs) / (kms / 1e3)
                                             / 1e12 / FP64_VALU_PEAK_TF, 4)
    return res


def hard_geometry(prob, C, local, dev, W_it, S_it, cols, cpu, o_means, seed=1000):
    """The north-star convergence target (max R-hat < 1.01) measured in the same run:
    one config-3 step under the reference's own hard-geometry profile
    (Tests/testGamma.R:45: adapt_delta 0.99, max_treedepth 12; the Shiny app's
    'adapt_delta' / 'max_treedepth' controls, ShinyInterface/server.R:97-100), timed
    like a headline step (inputs staged before the timer, synchronised both sides).
    The CPU rate is the headline leg's measured oracle gradient rate scaled by this
    step's gradients per post-warmup draw (per-gradient cost does not depend on the
    controls), so no second CPU run is needed."""
    import torch
    from fitoct_amd import Plan
    cfg = make_config(seed, C, 0, local, W_it, S_it, 0.99, 12)
    with Plan(prob, cfg) as pl:
        buf = torch.empty(pl.info["draws_bytes"] // 8, dtype=torch.float64, device=dev)
        stream = torch.cuda.current_stream(dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pl.run(d_draws=buf.data_ptr(), stream=stream.cuda_stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        out = pl.download()
    kms = out.kernel_ms
    lf = out.total_leapfrogs
    value = C * S_it / wall
    conv = convergence(out.draws, out.warmup_saved, cols)
    res = {"workload": (f"fitExpGP+horseshoe N={N_BINS} Nn={NN} {C} chains W={W_it} S={S_it} "
                        "adapt_delta=0.99 max_treedepth=12 (Tests/testGamma.R:45)"),
           "seed": seed, "value": round(value, 2), "unit": "draws/s",
           "ms_per_step": round(wall * 1e3, 2), "kernel_ms": round(kms, 2),
           "gradients_per_launch": lf,
           "gradients_per_iteration": round(lf / (C * (W_it + S_it)), 1),
           "roofline_frac": round(f_grad(N_BINS, NN) * lf / (kms / 1e3) / 1e12
                                  / FP64_VALU_PEAK_TF, 4),
           **conv}
    if cpu is not None:
        # draws/s of the CPU path at this profile: its gradient rate over this step's
        # gradients per post-warmup draw (warmup included, as for the GPU's value)
        cpu_value = cpu["lf_rate"] * C * S_it / lf
        res["cpu_baseline"] = {"value": round(cpu_value, 2), "unit": "draws/s",
                               "cores": cpu["cores"], "kind": cpu["kind"],
                               "value_node_est": round(cpu_value * cpu["host"]["node_cpus"]
                                                       / cpu["cores"], 2),
                               "sample": "the headline leg's oracle gradient rate "
                                         f"({cpu['lf_rate']:.3g} grad/s on {cpu['cores']} "
                                         f"threads) over this step's {lf / (C * S_it):.1f} "
                                         "gradients per post-warmup draw"}
        res["gpu_over_cpu"] = round(value / cpu_value, 1)
        res["gpu_over_cpu_node_est"] = round(value / res["cpu_baseline"]["value_node_est"], 2)
    if o_means is not None:
        g_means = np.nanmean(out.draws[:, out.warmup_saved:, :], axis=(0, 1))
        res["posterior_mean_relerr_vs_cpu"] = {
            n: round(float(abs(g_means[j] - o_means[j]) / abs(o_means[j])), 6)
            for j, n in enumerate(cols) if n.startswith("theta") or n in ("sigma", "br")}
    return res


def bench_batch(args, world, rank, local, dev, dist, backend, cdev, W_it, S_it, dev_list=()):
    """Config 5 (FitOCT.R batch mode): this rank's files in ONE batched launch
    (fitoct_batch_*); one gather of every rank's draws to rank 0 inside the step.
    With ``--devices N`` (one process) the batch runs over the C ABI's device list."""
    import torch
    from fitoct_amd import Batch, ExpGPProblem, SamplerConfig
    from fitoct_amd.stanfit import split_rhat_ess
    from fitoct_amd.synth import MODULATIONS, default_prior, synth_decay

    conf = CONFIGS[5]
    ndev = torch.cuda.device_count()
    t0, S0 = default_prior()
    from fitoct_amd.distributed import shard_range
    f_off, f_cnt = shard_range(conf["files"], world, rank)   # contiguous file blocks

    def file_problems(first, count):
        out = []
        for f in range(first, first + count):
            d = synth_decay(conf["N"], MODULATIONS[f % 4], 1234 + f)
            out.append(ExpGPProblem(d["x"], d["y"], d["uy"], dataType=2, Nn=NN,
                                    gridType="extremal", theta0=t0, Sigma0=S0,
                                    prior_type=conf["prior"]))
        return out
    files = list(range(f_off, f_off + f_cnt))
    probs = file_problems(f_off, f_cnt)
    C = args.chains or conf["chains"]
    n_units = len(dev_list) or world

    def batch_for(step, ps=probs, first=f_off, devs=dev_list):
        # file f's chains are global chains f*C + c (fitoct_amd.distributed.sample_batch_sharded)
        cfg = SamplerConfig(chains=C, warmup=W_it, samples=S_it, seed=2000 + step,
                            adapt_delta=0.8, max_treedepth=10, device=local,
                            chain_offset=first * C, devices=devs)
        return Batch(ps, cfg)

    stream = torch.cuda.current_stream(dev)
    bufs = {}

    def run_step(b):
        key = b.info["draws_bytes"]
        if key not in bufs:
            bufs[key] = torch.empty(key // 8, dtype=torch.float64, device=dev)
        buf = bufs[key]
        b.run(d_draws=buf.data_ptr(), stream=0 if dev_list else stream.cuda_stream)
        if world > 1:   # ragged file counts per rank: all_gather of sizes, then gather
            src = buf if backend == "nccl" else buf.cpu()
            n = torch.tensor([src.numel()], dtype=torch.int64, device=cdev)
            sizes = [torch.zeros_like(n) for _ in range(world)]
            dist.all_gather(sizes, n)
            m = int(max(int(x.item()) for x in sizes))
            pad = torch.zeros(m, dtype=torch.float64, device=src.device)
            pad[:src.numel()] = src
            gl = [torch.empty(m, dtype=torch.float64, device=src.device)
                  for _ in range(world)] if rank == 0 else None
            dist.gather(pad, gather_list=gl, dst=0)

    for w in range(args.warmup):
        with batch_for(-1 - w) as b:
            run_step(b)
    torch.cuda.synchronize()
    batches = [batch_for(s) for s in range(args.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t_0 = time.perf_counter()
    for b in batches:
        run_step(b)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t_0
    if dist is not None:
        t = torch.tensor([wall], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())

    last = batches[-1]
    outs = [last.download(p) for p in range(len(probs))]
    kernel_ms = float(np.mean([b.download(0, with_draws=False).kernel_ms for b in batches]))
    lf = sum(o.total_leapfrogs for o in outs)
    cols = probs[0].column_names()
    par = [j for j in range(7, len(cols))]
    rh_file = [max(split_rhat_ess(o.draws[:, o.warmup_saved:, j])[0] for j in par) for o in outs]
    ms_per_step = wall * 1e3 / args.steps
    draws_step = conf["files"] * C * S_it
    achieved = f_grad(conf["N"], NN) * lf / (kernel_ms / 1e3) / 1e12
    line = {
        "metric": "posterior draws/sec (all chains), config 5 (FitOCT.R batch mode)",
        "value": round(draws_step / (ms_per_step / 1e3), 2), "unit": "draws/s",
        "n_gpus": n_units, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 2), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (restated synthData.R, 4 modulations cycled over files)",
        "config": {"workload": f"FitOCT.R batch: {conf['files']} files x {C} chains, "
                               f"fitExpGP+{conf['prior']} N={conf['N']} Nn={NN} W={W_it} S={S_it}",
                   "files": conf["files"], "files_this_rank": len(files), "chains_per_file": C,
                   "parallelism": (f"files in contiguous blocks over {n_units} GPU(s), one "
                                   "launch per GPU" + (f" (device list {list(dev_list)}, one "
                                                       "process)" if dev_list else "")),
                   "route": ("device-list" if dev_list else
                             "torch.distributed" if world > 1 else "single-device")},
        "rhat_max_median_file": round(float(np.median(rh_file)), 4),
        "rhat_max_worst_file": round(float(np.max(rh_file)), 4),
        # the Shiny app paints R-hat >= 1.1 red (ShinyInterface/server.R:98-100); the C
        # oracle on the same 256 files gives 27 / 256 (tests/golden/batch_files.npz)
        "rhat_files_ge_1_1": round(float(np.mean(np.array(rh_file) >= 1.1)), 4),
        "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": FP64_VALU_PEAK_TF,
                     "unit": "TFLOP/s", "frac": round(achieved / FP64_VALU_PEAK_TF, 4),
                     "traffic": None, "kernel": "nuts_kernel (batched)",
                     "kernel_ms": round(kernel_ms, 2), "gradients_per_launch_rank0": lf},
    }
    traffic = load_traffic(line["config"]["workload"])
    if traffic:
        r = line["roofline"]
        r["traffic"] = traffic["bytes_per_launch"]
        r["hbm_gbs"] = round(traffic["bytes_per_launch"] / (kernel_ms / 1e3) / 1e9, 2)
        r["hbm_frac"] = round(r["hbm_gbs"] / HBM_PEAK_GBS, 5)
        r["traffic_source"] = traffic["source"]
    if rank == 0 and n_units == 1 and not args.no_cpu:
        cb = batch_cpu_baseline(file_problems, conf["files"], C, W_it, S_it, 2000 + args.steps - 1,
                                outs)
        line["posterior_mean_relerr_vs_cpu"] = cb.pop("relerr")
        line["cpu_baseline"] = cb
        line["gpu_over_cpu"] = round(line["value"] / cb["value"], 1)
    for b in batches:
        b.close()
    bufs.clear()
    if n_units == 1:
        # Config 5 scales strongly (256 files in total), and each GPU's share is an
        # independent launch: N GPUs take as long as 256/N files on one GPU (plus the
        # gather), which this GPU measures -- the floor being one file's slowest chain.
        line["strong_scaling_est"] = strong_scaling_est(
            lambda n: batch_for(0, file_problems(0, conf["files"] // n), 0),
            conf["files"], C * S_it, line["ms_per_step"])
    if world > 1 and not args.no_device_list:
        hb = dist.new_group(backend="gloo")   # host barrier: no collective kernel on the GPUs
        dist.barrier(group=hb)
        if rank == 0:
            try:   # a side measurement: it must not cost the main line
                every = file_problems(0, conf["files"])
                line["device_list"] = device_list_leg(
                    lambda step, devs: batch_for(step, every, 0, devs), _dl_devices(world, ndev),
                    conf["files"] // world * C * S_it, dev, f_grad(conf["N"], NN),
                    is_batch=True)
            except Exception as e:   # noqa: BLE001
                line["device_list"] = {"error": f"{type(e).__name__}: {e}"}
        dist.barrier(group=hb)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def batch_cpu_baseline(file_problems, files, C, W, S, seed, gpu_outs, budget_s=12.0):
    """Config 5's CPU path: the C oracle (one OpenMP thread per chain) on the SAME files,
    chains (global ids f*C + c), controls and seed as the last timed GPU step, so no
    scaling is needed: value = files done x C x S / wall.  Bounded: files are run
    ``share_cpus // C`` at a time from file 0 until ``budget_s`` has passed (the job's
    CPU share; the rest of the 256 files would run at the same rate).  Posterior means
    of theta, sigma and br per file against the GPU's same files: median and max of the
    relative difference over the files run (4 chains x 100 draws per side, so the
    figure includes both sides' Monte-Carlo error)."""
    from concurrent.futures import ThreadPoolExecutor

    from fitoct_amd import SamplerConfig
    from oracle import nuts_c
    hw = host_cpu_info()
    threads = hw["share_cpus"]
    conc = max(1, threads // C)

    def one(f):
        prob = file_problems(f, 1)[0]
        cfg = SamplerConfig(chains=C, chain_offset=f * C, warmup=W, samples=S, seed=seed,
                            adapt_delta=0.8, max_treedepth=10)
        o = nuts_c.sample(prob, cfg, nthreads=C)
        return f, o
    done = []
    t = time.perf_counter()
    with ThreadPoolExecutor(max_workers=conc) as ex:
        f = 0
        while f < files and (time.perf_counter() - t < budget_s or not done):
            done += list(ex.map(one, range(f, min(files, f + conc))))
            f += conc
    wall = time.perf_counter() - t
    cols = file_problems(0, 1)[0].column_names()
    names = [n for n in cols if n.startswith("theta") or n in ("sigma", "br")]
    rel = {n: [] for n in names}
    lf = 0
    for f, o in done:
        lf += int(o["leapfrogs"].sum())
        mc = np.nanmean(o["draws"][:, W:, :], axis=(0, 1))
        g = gpu_outs[f]
        mg = np.nanmean(g.draws[:, g.warmup_saved:, :], axis=(0, 1))
        for n in names:
            j = cols.index(n)
            rel[n].append(abs(mg[j] - mc[j]) / abs(mc[j]))
    value = len(done) * C * S / wall
    return {"value": round(value, 2), "unit": "draws/s", "cores": threads, "kind": "port",
            "value_node_est": round(value * hw["node_cpus"] / threads, 2), "host": hw,
            "sample": (f"C oracle NUTS on files 0..{len(done) - 1} of the {files} ({C} chains x "
                       f"({W} warmup + {S} draws) each, the same chain ids, controls and seed "
                       f"{seed} as the GPU's last step), {conc} files at a time x {C} threads "
                       f"on this job's {threads}-CPU share of a {hw['node_cpus']}-CPU node: "
                       f"{lf} gradients in {wall:.1f} s"),
            "wall_s": round(wall, 2), "files": len(done),
            "relerr": {"files": len(done),
                       "median": {n: round(float(np.median(v)), 6) for n, v in rel.items()},
                       "max": {n: round(float(np.max(v)), 6) for n, v in rel.items()}}}


def strong_scaling_est(make, files, draws_per_file, ms_1):
    """Per-GPU share of a strong-scaling run of `files` files on n GPUs, timed on this
    one GPU: a batch of files/n files (one untimed run, then one timed).  The
    estimate ignores the gather (a few MB per GPU over xGMI) and assumes the GPUs do
    not slow one another (independent launches, no collective during sampling)."""
    import torch
    out = []
    for n in (2, 4, 8):
        with make(n) as b:
            b.run()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            b.run()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
        out.append({"n_gpus": n, "files_per_gpu": files // n, "ms_per_step_est": round(ms, 2),
                    "value_est": round(files * draws_per_file / (ms / 1e3), 2),
                    "efficiency_est": round(ms_1 / (n * ms), 4)})
    return out


if __name__ == "__main__":
    main()
