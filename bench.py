"""bench.py — Gibbs sweeps/s of the MI355X sampler (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[3], one shard per GPU): synthetic data
N = 1,000,000 customers, V = 4 views, D = 128 dims, K = 64 generating
clusters (per-view K_v = 64, 32, 16, 8), fp64; one independent chain per
GPU (chain id = rank, weak scaling).  A "step" is one full parallel sweep
(z-resample of all N customers + birth resolution + commit + stats rebuild +
hyperparameter MH).  The chain is warm-started at the generating partition so
the measured state has ~K tables (the reference's cold initialisation has a
long transient); every timed sweep does the complete work.

Multi-GPU: launched by torch.distributed.run, one process per GPU, chains
shard embarrassingly (no collective in the sweep); the timed region is
bracketed by barrier + device sync and the max over ranks is reported.

Output: one JSON line on rank 0 (driver contract), including the roofline of
the dominant kernel (zresample) measured with HIP events on the sampler's
stream, and a CPU baseline (the oracle's restatement of the same chain, one
full sweep on one host core).  With N = 1 it also reports (key `extra`) the
GPU on the north_star literal (D = 1) and configs[1], the exact schedule on
configs[0], a cold start on configs[1], and the reference's algorithm
(oracle ExactSampler, libm) on the host at the north_star literal.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multiview-clustering_amd")]

# Every GPU leg runs in a child process (child_leg) with the caller's
# GPU_MAX_HW_QUEUES (HIP's default of 4 when unset): the multi-chain legs use
# the chain-batched repair, which needs no hardware queue per chain
# (DESIGN.md §7).  The value is recorded before the library loads.
CALLER_HW_QUEUES = os.environ.get("GPU_MAX_HW_QUEUES")

import numpy as np  # noqa: E402

CONFIGS = {
    # name: (N, V, D, K, description)
    "c4": (1_000_000, 4, 128, 64, "BASELINE configs[3] shard: synthetic N=1M V=4 D=128 K=64, 1 chain/GPU"),
    "c2": (100_000, 2, 64, 16, "BASELINE configs[1]: synthetic N=100k V=2 D=64 K=16, 1 chain"),
    "ns": (1_000_000, 4, 1, 64, "north_star literal: synthetic N=1M V=4 D=1 K=64, 1 chain/GPU"),
    "c5": (10_000_000, 8, 256, 256, "BASELINE configs[4]: synthetic N=10M V=8 D=256 K=256 fp64 (y generated on the "
                                    "device: 164 GB), 1 chain, MFMA dish-block producer"),
}
PEAK_HBM_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_F64_TFLOPS = 78.6       # fp64 MFMA / vector dense peak (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=int, default=1999)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--shard", action="store_true",
                    help="N > 1: ONE chain split over the N GPUs (within-chain N-sharding of phase A, an RCCL "
                         "all-gather of the choices per sweep; strong scaling) instead of one chain per GPU")
    ap.add_argument("--leg", default=None, help=argparse.SUPPRESS)   # child_leg: run one multi-chain leg, print it
    ap.add_argument("--leg-device", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the extra lines (other configs, exact schedule, cold start, reference CPU)")
    return ap.parse_args()


def warm_state(z, V, K):
    """Generating partition: table t = global cluster t, dish_v(t) = t mod K_v."""
    uniq = np.unique(z)
    remap = np.full(int(z.max()) + 1, -1, dtype=np.int64)
    remap[uniq] = np.arange(uniq.size)
    table_of = remap[z].astype(np.int32)
    dish = np.stack([uniq % max(1, K // (2 ** v)) for v in range(V)]).astype(np.int32)
    hyper = np.concatenate([np.full(V, 1.69), np.ones(V), np.full(V, 0.5), [1.0, 0.6]])
    return table_of, dish, hyper


def measured_traffic(config):
    """HBM bytes per z-resample pass from the committed rocprofv3 PMC summary
    (scripts/gpu_pmc_z.sh -> profiles/pmc_traffic.json), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
        return t.get(config, {}).get("bytes_per_pass")
    except (OSError, ValueError):
        return None


def host_cpu():
    """The host CPU model and core count (lscpu 'Model name', os.cpu_count)."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"model": model, "nproc": os.cpu_count()}


def cpu_baseline(y, z, V, K, D, seed, budget_s=30.0):
    """The oracle's restatement of the same chain (SeqSampler: the reference's
    sequential schedule with this build's D-dim conditional and counters;
    oracle/mvc_oracle.cpp), one full sweep over all N customers from the same
    warm state, on one host core (one chain -> min(chains, nproc) = 1 core).
    A 2000-customer probe predicts the sweep; only if it would exceed
    budget_s does it time a prefix and extrapolate (said in `sample`)."""
    from oracle import oracle as O
    N = y.shape[1]
    m = min(2000, N)
    t0 = time.perf_counter()
    O.run(np.ascontiguousarray(y[:, :m]), 1, 0, 1, seed, chain=0, mode=O.PARALLEL, state=warm_state(z[:m], V, K))
    per = (time.perf_counter() - t0) / m
    n_sample = N if per * N <= budget_s else int(max(m, budget_s / max(per, 1e-9)))
    ys = np.ascontiguousarray(y[:, :n_sample])
    st = warm_state(z[:n_sample], V, K)
    t0 = time.perf_counter()
    O.run(ys, 1, 0, 1, seed, chain=0, mode=O.PARALLEL, state=st)
    dt = time.perf_counter() - t0
    sweeps_per_s = 1.0 / (dt * (N / n_sample))
    what = (f"1 full sweep over all {N} customers, {dt:.2f} s" if n_sample == N else
            f"1 sweep over the first {n_sample} of {N} customers, {dt:.2f} s, extrapolated linearly to N")
    return {"value": sweeps_per_s, "unit": "sweeps/s", "cores": 1, "kind": "port",
            "host": host_cpu(),
            "sample": f"oracle SeqSampler (the sequential schedule the GPU runs; oracle/mvc_oracle.cpp, g++ -O2, "
                      f"portable math), same warm state and data: {what}"}


def reference_schedule_cpu(seed, budget_s=20.0):
    """The reference's own algorithm (oracle ExactSampler<LibmMath>: a
    line-by-line restatement of multiview_gibbs.cpp / multiview_utils.cpp /
    multiview_hyper.cpp with glibc libm, D = 1) at the north_star literal
    (N = 1M, V = 4, K = 64, D = 1), warm start at the generating partition,
    one full sweep on one core (one chain)."""
    from oracle import oracle as O
    from mvc_amd import data
    N, V, D, K, desc = CONFIGS["ns"]
    y, z = data.synthetic(N, V, D, K, seed=seed)
    y2 = np.ascontiguousarray(y[:, :, 0])
    m = 20000
    t0 = time.perf_counter()
    O.run(np.ascontiguousarray(y2[:, :m]), 1, 0, 1, seed, chain=0, mode=O.EXACT, math=O.LIBM,
          state=warm_state(z[:m], V, K))
    per = (time.perf_counter() - t0) / m
    n_sample = N if per * N <= budget_s else int(max(m, budget_s / max(per, 1e-9)))
    t0 = time.perf_counter()
    O.run(np.ascontiguousarray(y2[:, :n_sample]), 1, 0, 1, seed, chain=0, mode=O.EXACT, math=O.LIBM,
          state=warm_state(z[:n_sample], V, K))
    dt = time.perf_counter() - t0
    return {"workload": desc, "value": 1.0 / (dt * (N / n_sample)), "unit": "sweeps/s", "cores": 1,
            "kind": "reference-algorithm restatement (oracle ExactSampler<LibmMath>)", "host": host_cpu(),
            "sample": (f"1 full sweep over all {N} customers, {dt:.2f} s" if n_sample == N else
                       f"1 sweep over the first {n_sample} of {N} customers, {dt:.2f} s, extrapolated to N")}


def gpu_line(config, seed, device, steps=10, warmup=3):
    """sweeps/s of the GPU (parallel-mode handle, the sequential schedule) on
    another BASELINE config, warm start at the generating partition."""
    from mvc_amd import data
    from mvc_amd.sampler import Sampler
    N, V, D, K, desc = CONFIGS[config]
    y, z = data.synthetic(N, V, D, K, seed=seed)
    s = Sampler(y, seed=seed, mode="parallel", device=device)
    s.set_state(*warm_state(z, V, K))
    s.sweep(warmup)
    s.synchronize()
    t0 = time.perf_counter()
    s.sweep(steps)
    s.synchronize()
    dt = time.perf_counter() - t0
    rep = s.repair_stats()
    s.close()
    return {"workload": desc, "value": round(steps / dt, 3), "unit": "sweeps/s", "steps": steps,
            "moves_last_sweep": rep["moves"]}


def gpu_chains_line(config, seed, device, chains=64, sweeps=1):
    """Several chains of one config on one GPU at once (parallel-mode ChainSet,
    the data shared; the chain-batched repair: one block per chain in each
    repair launch), warm start at the generating partition:
    aggregate chain-sweeps/s, with HIP's default hardware queues."""
    from mvc_amd import data
    from mvc_amd.sampler import Sampler
    N, V, D, K, desc = CONFIGS[config]
    y, z = data.synthetic(N, V, D, K, seed=seed)
    st = warm_state(z, V, K)
    s = Sampler(y, seed=seed, mode="parallel", n_chains=chains, device=device)
    for c in range(chains):
        s.set_state(*st, chain=c)
    s.synchronize()
    t0 = time.perf_counter()
    s.sweep(sweeps)
    s.synchronize()
    dt = time.perf_counter() - t0
    s.close()
    return {"workload": desc.replace("1 chain/GPU", f"{chains} chains on 1 GPU at once"), "chains": chains,
            "sweeps": sweeps, "value": round(chains * sweeps / dt, 3), "unit": "chain-sweeps/s",
            "s_per_sweep_all_chains": round(dt / sweeps, 2)}


def gpu_exact_line(seed, device, chains=2048, sweeps=200):
    """BASELINE configs[0] (the New_Simulation.R problem, N = 500, V = 2, K = 3,
    200 sweeps) on the exact schedule (mode E: the reference's arithmetic,
    one wavefront per chain): `chains` independent chains in one handle."""
    from mvc_amd import data
    from mvc_amd.sampler import Sampler
    y, _ = data.config1(seed=1)
    s = Sampler(y, seed=seed, mode="exact", n_chains=chains, device=device)
    s.synchronize()
    t0 = time.perf_counter()
    s.sweep(sweeps)
    s.synchronize()
    dt = time.perf_counter() - t0
    s.close()
    return {"workload": "BASELINE configs[0]: New_Simulation shape N=500 V=2 K=3 (D=1), cold start, exact schedule",
            "chains": chains, "sweeps": sweeps, "value": round(chains * sweeps / dt, 1),
            "unit": "chain-sweeps/s", "per_chain_sweeps_per_s": round(sweeps / dt, 2)}


def config5_line(seed, device, steps=3, warmup=1):
    """BASELINE configs[4] at its full size: N = 10M, V = 8, D = 256, K = 256
    (164 GB of y, generated on the device by mvc_sampler_create_synthetic;
    the host never holds it), warm start at the generating partition.
    sweeps/s plus the z-resample pass against both roofs: MFMA fp64 (2 N D
    sum K_v flops, AI ~ 64 flop/B: the binding roof) and HBM (the algorithmic
    N (8 V D + 8) bytes)."""
    from mvc_amd.sampler import Sampler
    N, V, D, K, desc = CONFIGS["c5"]
    t0 = time.perf_counter()
    s, z = Sampler.synthetic(N, V, D, K, data_seed=seed, seed=seed, device=device, timing="coarse")
    s.set_state(*warm_state(z, V, K))
    s.sweep(warmup)
    s.synchronize()
    setup = time.perf_counter() - t0
    s.reset_timers()
    t1 = time.perf_counter()
    s.sweep(steps)
    s.synchronize()
    dt = time.perf_counter() - t1
    kms, kcnt = s.kernel_time("zresample")
    kd = s.dish_counts()
    rep = s.repair_stats()
    zp = s.zpath()
    s.close()
    pass_s = kms / max(1, kcnt) / 1e3
    flops = 2.0 * N * D * float(kd.sum())
    byts = N * (8 * V * D + 8)
    return {"workload": desc, "value": round(steps / dt, 4), "unit": "sweeps/s", "steps": steps,
            "ms_per_sweep": round(1e3 * dt / steps, 2), "setup_s": round(setup, 1), "pass_ms": round(pass_s * 1e3, 2),
            "mfma_tflops": round(flops / pass_s / 1e12, 2), "mfma_frac": round(flops / pass_s / 1e12 / PEAK_F64_TFLOPS, 4),
            "hbm_gbs": round(byts / pass_s / 1e9, 1), "hbm_frac": round(byts / pass_s / 1e9 / PEAK_HBM_GBS, 4),
            "bound": "mfma", "dishes": kd.tolist(), "moves_last_sweep": rep["moves"],
            "producer": "mfma-dish-blocks" if zp & 64 else "other"}


def newsim_call_line(seed, device, M=10000, M_short=2000):
    """The reference's own caller (New_Simulation.R:123-133: N = 200, V = 5,
    M = 10,000, burn-in 9,000, thin 1, the data of :47-60) through the
    drop-in entry point mvc_run, in both schedules, against the reference's
    algorithm on one host core (oracle ExactSampler<LibmMath>).  The parallel
    schedule (the drop-in's default) runs the whole call; the exact schedule
    and the host run M_short sweeps (their per-sweep cost is flat after the
    first few hundred sweeps) and are reported as sweeps/s."""
    import mvc_amd
    from mvc_amd import data
    y, _ = data.new_simulation(seed)
    out = {"workload": "New_Simulation.R call: N=200 V=5 M=10000 burn_in=9000 thin=1, one chain"}
    t0 = time.perf_counter()
    mvc_amd.run_gibbs_cpp(y, M, M - 1000, 1, seed=seed, mode="parallel", device=device, quiet=True)
    dt = time.perf_counter() - t0
    out["parallel_gpu"] = {"sweeps": M, "s": round(dt, 2), "sweeps_per_s": round(M / dt, 1)}
    t0 = time.perf_counter()
    mvc_amd.run_gibbs_cpp(y, M_short, M_short - 200, 1, seed=seed, mode="exact", device=device, quiet=True)
    dt = time.perf_counter() - t0
    out["exact_gpu"] = {"sweeps": M_short, "s": round(dt, 2), "sweeps_per_s": round(M_short / dt, 1)}
    out["default_mode"] = "parallel"
    return out


def newsim_chains_line(seed, device):
    """The same call with several chains per call (MVC_CHAINS in the drop-in):
    aggregate chain-sweeps/s, parallel schedule 16 chains, exact 2048 (one
    wavefront each, 8 per CU); for the exact schedule also the sweeps alone,
    without mvc_run's per-sample bookkeeping, at 2048 and 4096 chains."""
    import mvc_amd
    from mvc_amd import data
    from mvc_amd.sampler import Sampler
    y, _ = data.new_simulation(seed)
    out = {}
    for mode, C, Mc in (("parallel", 16, 1000), ("exact", 2048, 500)):
        tm = {}
        t0 = time.perf_counter()
        mvc_amd.run_gibbs_cpp(y, Mc, Mc // 2, 1, seed=seed, mode=mode, n_chains=C, device=device, quiet=True,
                              timing=tm)
        dt = time.perf_counter() - t0
        # the library call (mvc_run: every chain's samples saved on the host, as the reference's
        # C++ returns them) timed alone; the Python lists built from them are reported beside it
        out[f"{mode}_gpu_{C}chains"] = {"chains": C, "sweeps": Mc, "s": round(tm["mvc_run_s"], 2),
                                        "chain_sweeps_per_s": round(C * Mc / tm["mvc_run_s"], 1),
                                        "python_result_lists_s": round(dt - tm["mvc_run_s"], 2)}
    Mc = 500
    for C in (2048, 4096):   # 8 chains per CU resident (2 per SIMD): 4096 is two full rounds
        s = Sampler(y, seed=seed, mode="exact", n_chains=C, device=device)
        s.sweep(Mc // 2)                      # past the cold-start transient
        s.synchronize()
        t0 = time.perf_counter()
        s.sweep(Mc)
        s.synchronize()
        dt = time.perf_counter() - t0
        s.close()
        out[f"exact_gpu_{C}chains_sweeps_only"] = {"chains": C, "sweeps": Mc, "s": round(dt, 2),
                                                   "chain_sweeps_per_s": round(C * Mc / dt, 1)}
    return out


CHILD_LEGS = {
    # name: function(seed, device) -> dict
    "north_star_literal_gpu": lambda seed, dev: gpu_line("ns", seed, dev, 1, 0),
    "north_star_literal_gpu_64chains": lambda seed, dev: gpu_chains_line("ns", seed, dev, chains=64),
    "configs1_gpu": lambda seed, dev: gpu_line("c2", seed, dev),
    "configs4_full_gpu": lambda seed, dev: config5_line(seed, dev),
    "exact_schedule_gpu": lambda seed, dev: gpu_exact_line(seed, dev),
    "newsim_call": lambda seed, dev: newsim_call_line(seed, dev),
    "newsim_chains": lambda seed, dev: newsim_chains_line(seed, dev),
    "cold_start_gpu": lambda seed, dev: cold_start(seed, dev),
}


def child_leg(name, seed, device, timeout=300):
    """Run CHILD_LEGS[name] in a child process (its own HIP runtime).  Never raises: a leg that
    fails, faults or times out is recorded as {"error": ...}, so no extra
    leg can take the headline line with it."""
    import subprocess
    env = dict(os.environ)
    env["GPU_MAX_HW_QUEUES"] = CALLER_HW_QUEUES if CALLER_HW_QUEUES is not None else "4"
    t = time.perf_counter()
    try:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--leg", name, "--seed", str(seed),
                            "--leg-device", str(device)], env=env, capture_output=True, text=True, timeout=timeout)
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {timeout} s"}
    finally:
        print(f"bench: {name} {time.perf_counter() - t:.1f} s", file=sys.stderr, flush=True)
    if r.returncode != 0:
        return {"error": f"exit {r.returncode}: {r.stderr.strip()[-600:]}"}
    try:
        return json.loads(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return {"error": "no JSON line from the leg: " + r.stdout[-300:]}


def newsim_call_cpu(seed, M_short=2000):
    """CPU baseline of newsim_call_line: the reference's algorithm (oracle
    ExactSampler<LibmMath>, the line-by-line restatement) on one host core,
    M_short sweeps of the same call."""
    from mvc_amd import data
    from oracle import oracle as O
    y, _ = data.new_simulation(seed)
    t0 = time.perf_counter()
    O.run(y, M_short, M_short - 200, 1, seed=seed, mode=O.EXACT, math=O.LIBM)
    dt = time.perf_counter() - t0
    return {"sweeps": M_short, "s": round(dt, 2), "sweeps_per_s": round(M_short / dt, 1), "cores": 1,
            "kind": "reference-algorithm restatement (oracle ExactSampler<LibmMath>)", "host": host_cpu()}


def cold_start(seed, device, sweeps=4):
    """BASELINE configs[1] (N = 100k, V = 2, D = 64, K = 16) from the
    reference's initialisation (4 tables, 2 dishes per view,
    multiview_gibbs.cpp:12-103): seconds, tables and movers per sweep."""
    from mvc_amd import data
    from mvc_amd.sampler import Sampler
    N, V, D, K, desc = CONFIGS["c2"]
    y, _ = data.synthetic(N, V, D, K, seed=seed)
    s = Sampler(y, seed=seed, mode="parallel", device=device)
    s.synchronize()
    rows = []
    for _ in range(sweeps):
        t0 = time.perf_counter()
        s.sweep(1)
        s.synchronize()
        dt = time.perf_counter() - t0
        rep = s.repair_stats()
        rows.append({"s": round(dt, 4), "T": int(s.state()[1].shape[1]), "moves": rep["moves"],
                     "births": rep["births"]})
    s.close()
    return {"workload": desc + ", cold start", "sweeps": rows}


def main():
    args = parse()
    if args.leg:   # a child_leg process: one multi-chain leg, one JSON line
        print(json.dumps(CHILD_LEGS[args.leg](args.seed, args.leg_device)), flush=True)
        return
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    N, V, D, K, desc = CONFIGS[args.config]

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        # RCCL over xGMI; MVC_BENCH_BACKEND=gloo only to rehearse several ranks on one GPU
        dist.init_process_group(os.environ.get("MVC_BENCH_BACKEND", "nccl"))

    def barrier_sync():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    from mvc_amd import data
    from mvc_amd.sampler import Sampler

    t_gen = time.perf_counter()
    shard = args.shard and world > 1
    if args.config == "c5":   # 164 GB of y: generated on the device, never on the host
        y = None
        s, z = Sampler.synthetic(N, V, D, K, data_seed=args.seed, seed=args.seed, first_chain=0 if shard else rank,
                                 device=local, timing="coarse")
    else:
        y, z = data.synthetic(N, V, D, K, seed=args.seed)
    t_gen = time.perf_counter() - t_gen
    # coarse timing in the timed region: HIP events around the z-resample pass
    # (the roofline) and the sweep only; the per-phase breakdown is taken on
    # extra sweeps after the timed region (each event pair idles the GPU ~5 us)
    if y is not None:
        s = Sampler(y, seed=args.seed, mode="parallel", first_chain=0 if shard else rank, device=local,
                    timing="coarse")
    s.set_state(*warm_state(z, V, K))
    if shard:   # every rank holds the whole chain; phase A split, choices all-gathered
        from mvc_amd.dist import ShardExchange
        s.set_shard(rank, world, ShardExchange(N, rank, world, device=local))
    s.sweep(args.warmup)
    s.synchronize()
    s.reset_timers()
    print(f"bench: data {t_gen:.1f} s, warm-up done", file=sys.stderr, flush=True)

    barrier_sync()
    t0 = time.perf_counter()
    s.sweep(args.steps)
    s.synchronize()
    barrier_sync()
    elapsed = time.perf_counter() - t0

    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    kms, kcnt = s.kernel_time("zresample")
    sweep_ms, _ = s.kernel_time("sweep")
    # posterior-mean accumulators over 10 more saved sweeps (after the timed
    # region), reduced across ranks with R-hat
    from mvc_amd import dist as mdist
    s.set_timing(False)
    cstats = mdist.ChainStats(3 * V + 2)
    for _ in range(10):
        s.sweep(1)
        _, _, h = s.state()
        hv = np.concatenate([h["alpha_v"], h["sigma_v"], h["tau_v"], [h["alpha_global"], h["sigma_global"]]])
        if not (shard and rank != 0):   # a sharded chain is counted once
            cstats.add(0, hv)
    n_detail = 3
    s.set_timing(True)
    s.reset_timers()
    s.sweep(n_detail)
    s.synchronize()
    parts = {k: s.kernel_time(k)[0] / n_detail
             for k in ("zresample", "lp", "draw", "repair", "hyper")}
    repair = s.repair_stats()
    kdish = s.dish_counts()
    _, dish_now, hyper_now = s.state()
    T = dish_now.shape[1]
    zpath = s.zpath()
    s.close()

    # the cross-chain reduce of the hyperparameter accumulators (one
    # all-reduce over RCCL, outside the timed region; reported, never fed
    # back: DESIGN.md §7)
    red = cstats.reduce(device=f"cuda:{local}" if dist is not None else None)
    pooled_mean = red["mean"]

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    k_avg_s = (kms / max(1, kcnt)) / 1e3
    # customers of rank 0's pass: the whole chain, or its shard (--shard)
    from mvc_amd.dist import shard_len
    n_pass = min(N, shard_len(N, world)) if shard else N
    bytes_alg = n_pass * (8 * V * D + 8)                 # y read once + z read + choice write
    flops_alg = 2.0 * n_pass * float(kdish.sum()) * D    # G = Y S1^T per view (MFMA fp64)
    hbm_gbs = bytes_alg / k_avg_s / 1e9
    tflops = flops_alg / k_avg_s / 1e12
    ridge = PEAK_F64_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9)
    traffic = measured_traffic(args.config)
    roof = ({"bound": "mfma", "achieved": round(tflops, 3), "peak": PEAK_F64_TFLOPS, "unit": "TFLOP/s",
             "frac": round(tflops / PEAK_F64_TFLOPS, 4), "traffic": traffic}
            if flops_alg / bytes_alg > ridge else
            {"bound": "hbm", "achieved": round(hbm_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
             "frac": round(hbm_gbs / PEAK_HBM_GBS, 4), "traffic": traffic})
    value = (1 if shard else world) * args.steps / elapsed
    out = {
        "metric": "Gibbs sweeps/sec (N×V×K) at 1/2/4/8 MI355X; % HBM roofline",
        "value": round(value, 4),
        "unit": "sweeps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "strong" if shard else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": desc, "N": N, "V": V, "D": D, "K": K, "chains": 1 if shard else world,
                   "schedule": "sequential (reference) schedule, data-parallel pass + in-order repair (DESIGN.md §4.8)",
                   "parallelism": f"shard{world}" if shard else f"chains{world}",
                   "tables_at_end": int(T), "dishes_at_end": kdish.tolist()},
        "roofline": roof,
        "hbm": {"pass": "z-resample (lp producer + draw, DESIGN.md §5)", "achieved_gbs": round(hbm_gbs, 1),
                "peak_gbs": PEAK_HBM_GBS, "frac": round(hbm_gbs / PEAK_HBM_GBS, 4),
                "mfma_tflops": round(tflops, 3), "mfma_frac": round(tflops / PEAK_F64_TFLOPS, 4),
                "arith_intensity": round(flops_alg / bytes_alg, 3), "ridge": round(ridge, 3),
                "bytes_per_launch": bytes_alg, "flops_per_launch": flops_alg, "pass_ms": round(k_avg_s * 1e3, 4),
                "lp_producer": ("mfma-all-views" if zpath & 16
                                else "mfma" if (zpath & 3) == 2 else "mfma-dish-blocks" if zpath & 64
                                else "generic"),
                "draw": "registers" if zpath & 4 else "lds-checkpoints"},
        "hyper_pooled": {"chains": red["chains"], "draws": red["count"],
                         "alpha_global": round(float(pooled_mean[-2]), 6),
                         "sigma_global": round(float(pooled_mean[-1]), 6),
                         "rhat_max": None if red["rhat"] is None else round(float(np.nanmax(red["rhat"])), 4)},
        "nvk_sweeps_per_s": round(value * N * V * K, 1),
        "kernel_ms_per_sweep": {k: round(v, 4) for k, v in parts.items()},
        "repair_last_sweep": repair,
        "kernel_ms_note": "per-phase HIP-event times from 3 sweeps after the timed region",
        "data_gen_s": round(t_gen, 2),
    }
    def leg(name, fn, *a):
        """A host-side leg (CPU only); an exception is recorded, not raised."""
        t = time.perf_counter()
        try:
            r = fn(*a)
        except Exception as e:   # noqa: BLE001 -- the headline must survive any extra
            r = {"error": f"{type(e).__name__}: {e}"[:600]}
        print(f"bench: {name} {time.perf_counter() - t:.1f} s", file=sys.stderr, flush=True)
        return r

    # the headline's CPU baseline first (host only), then the extras
    if world == 1 and not args.no_cpu_baseline and y is not None:
        out["cpu_baseline"] = leg("cpu_baseline", cpu_baseline, y, z, V, K, D, args.seed)
    if world == 1 and not args.no_extras:
        # other BASELINE configs and schedules, after the timed region (rank 0,
        # N = 1), each GPU leg in its own process so that no failure there can
        # reach this process's line
        ex = out["extra"] = {}
        for name in CHILD_LEGS:
            if name == "newsim_chains":
                continue
            ex[name] = child_leg(name, args.seed, local)
        ex["newsim_call"] = {**ex.get("newsim_call", {}), "chains": child_leg("newsim_chains", args.seed, local)}
        if not args.no_cpu_baseline:
            ex["reference_schedule_cpu"] = leg("reference_schedule_cpu", reference_schedule_cpu, args.seed)
            ex["newsim_call"]["reference_cpu_1core"] = leg("newsim_call_cpu", newsim_call_cpu, args.seed)
            try:   # the chains' comparator: min(chains, nproc) host cores, one chain each
                ch = ex["north_star_literal_gpu_64chains"]
                ref1 = ex["reference_schedule_cpu"]["value"]
                cores = min(ch["chains"], os.cpu_count() or 1)
                ch["cpu_cores_compared"] = cores
                ch["reference_cpu_same_cores"] = round(cores * ref1, 3)
                ch["vs_reference_cpu_same_cores"] = round(ch["value"] / (cores * ref1), 3)
            except (KeyError, TypeError):
                pass
            try:
                r1 = ex["newsim_call"]["reference_cpu_1core"]["sweeps_per_s"]
                for key, row in ex["newsim_call"]["chains"].items():
                    if isinstance(row, dict) and "chains" in row:
                        cores = min(row["chains"], os.cpu_count() or 1)
                        row["cpu_cores_compared"] = cores
                        row["vs_reference_cpu_same_cores"] = round(row["chain_sweeps_per_s"] / (cores * r1), 3)
            except (KeyError, TypeError):
                pass
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
