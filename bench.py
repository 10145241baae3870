"""Headline benchmark: whole-node env-steps/s of the MuZero-Breakout acting loop.

Workload (BASELINE.json north_star): 4096 parallel envs per GPU x 50 MCTS sims on one MI355X
(= config 4's per-GPU share; --envs 1024 is config 2), random-init reference-architecture nets
(state_dict format, seeded), bf16 on MFMA.
One "step" = one acting step over all envs of a GPU: rep-input assembly ->
representation -> 50 x (select, dynamics, prediction, backup) -> sampling -> env step
+ render + history + trajectory record; every RECORD_K steps the records are gathered
(RCCL gather to rank 0 for N>1) into rank 0's pinned host buffer (the replay-buffer sink).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       N>1 either under python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ... (WORLD_SIZE must
       equal N), or plain `python bench.py --gpus N`, which starts that torchrun as a child process itself.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md chip table)
RECORD_K = 16


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU (north_star: 4096)")
    ap.add_argument("--sims", type=int, default=50)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--dyn-dtype", default=None, choices=[None, "fp16"], help="fp16 dynamics net (config 5)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-envs", type=int, default=768,
                    help="bounded CPU sample (cpu_baseline + match rate): ~20 s of the CPU port on 16 host cores")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of HIP-graph replay")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the f32 parity-path replay of the first timed step (full-batch visit-count match)")
    ap.add_argument("--learner-streams", type=int, default=2, choices=[1, 2],
                    help="learner: 2 = prediction nets on a side stream beside the dynamics chain")
    ap.add_argument("--tower-variant", type=int, default=0, help="tower kernel (mzba_tower_set_variant; 0 = by batch)")
    ap.add_argument("--workload", default="acting", choices=["acting", "env", "learner", "selfcheck"],
                    help="acting: the whole acting loop (headline); env: env step + render + frame stack only "
                         "(configs 1/3, HBM roofline)")
    ap.add_argument("--height", type=int, default=None, help="env workload frame height (default 84)")
    ap.add_argument("--width", type=int, default=None, help="env workload frame width (default 84)")
    ap.add_argument("--hist", type=int, default=4, help="env workload frame-stack length")
    ap.add_argument("--minibatch", type=int, default=512, help="learner workload minibatch (config.yaml:7)")
    ap.add_argument("--parity-envs", type=int, default=512,
                    help="config 3 geometry: envs of the f32 parity-path replay (the first ones of the batch)")
    ap.add_argument("--halo-form", type=int, default=None, choices=[0, 1, 2],
                    help="conv_halo pixels per workgroup (mzba_conv_halo_set_form; default: the library's)")
    ap.add_argument("--no-halo", action="store_true",
                    help="A/B: large-image 3x3 convs on conv_big_bf16_kernel instead of the halo-tiled conv_halo_kernel")
    ap.add_argument("--pow-threads", type=int, default=1,
                    help="intra-op threads of the reference process whose temperature pow the sampling reproduces "
                         "(splits torch's pow into per-thread chunks from 3 x global envs >= 32768 on)")
    return ap.parse_args()


def env_bytes(H, W):
    """SURVEY §8(d) algorithmic HBM bytes per env-step: the H*W uint8 frame write, the compact
    state read + write (2 x 16 B), the action (8 B) and reward/done/valid (8 B)."""
    return H * W + 2 * 16 + 8 + 8


def run_env(args, world, rank, local):
    """Configs 1/3: B envs x (step + render + frame-stack push) per step, no search.
    `value` = env-steps/s over all ranks; roofline = algorithmic bytes / kernel time vs HBM."""
    sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
    from mzba.config import default_config
    from mzba.env import CompactBreakout
    from mzba import _lib as L
    H, W = args.height or 84, args.width or 84
    B = args.envs
    cfg = default_config()
    dev = torch.device(f"cuda:{local}")
    env = CompactBreakout(cfg["environment"], B, args.hist, H, W, seed=args.seed, env_offset=rank * B, device=dev)
    env.reset(0)
    g = torch.Generator(device=dev).manual_seed(args.seed + rank)
    acts = torch.randint(0, 3, (args.warmup + args.steps, B), device=dev, generator=g)
    for i in range(args.warmup):
        env.step(acts[i], i == 0)
    # the K timed steps (one mzba_env_step_compact launch each) replay as one HIP graph, as the
    # acting loop does: eager ctypes launches from Python (~20 us each) would be the bound
    stream = torch.cuda.Stream(device=dev)
    stream.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        with torch.cuda.graph(graph, stream=stream):
            for i in range(args.steps):
                env.step(acts[args.warmup + i], False)
        graph.replay()  # untimed: one pass of the captured steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        ev[0][0].record(stream)
        graph.replay()
        ev[0][1].record(stream)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    kms = ev[0][0].elapsed_time(ev[0][1]) / args.steps  # per launch, inter-launch gaps included
    achieved = B * env_bytes(H, W) / (kms * 1e-3) / 1e9
    traffic = None  # PMC bytes per launch (tools/gpu_round.sh), when measured for this geometry
    tpath = os.path.join(ROOT, "profiles", "env_hbm_traffic.json")
    if os.path.exists(tpath):
        tj = json.load(open(tpath))
        if (tj.get("envs"), tj.get("H"), tj.get("W")) == (B, H, W) and tj.get("write_bytes") is not None:
            traffic = tj["write_bytes"] + (tj.get("fetch_bytes") or 0)
    # the env kernel's own duration (rocprofv3 kernel trace of this geometry, profiles/env_kernel_time.json): the
    # event-timed figure above includes whatever separates consecutive graph-replayed launches
    ktimed = None
    kpath = os.path.join(ROOT, "profiles", "env_kernel_time.json")
    if os.path.exists(kpath):
        for e in json.load(open(kpath)):
            if (e["envs"], e["H"], e["W"], e["hist"]) == (B, H, W, args.hist):
                a_k = B * env_bytes(H, W) / (e["avg_ns"] * 1e-9) / 1e9
                ktimed = {"avg_kernel_ms": e["avg_ns"] * 1e-6, "achieved": a_k, "frac": a_k / 8000.0, "source": e["source"]}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        from oracle.env import BreakoutEnvOracle, convert_to_grayscale
        nb = min(B, 256)
        e = BreakoutEnvOracle({**cfg["environment"], "n_parallel": nb})
        e.height, e.width = H, W
        s, _ = e.reset(e.reset_params(args.seed, 0))
        done = np.zeros(nb, dtype=bool)
        rng = np.random.default_rng(args.seed)
        n, c0 = 0, time.perf_counter()
        while time.perf_counter() - c0 < 10.0 and n < 2000:
            s, r, done, v = e.step(s, rng.integers(0, 3, nb), done)
            convert_to_grayscale(s)
            n += 1
        cs = time.perf_counter() - c0
        cpu = {"value": nb * n / cs, "unit": "env-steps/s", "cores": 1, "kind": "port",
               "sample": f"oracle numpy env (batched like parallel_breakout.py) + grayscale, {nb} envs x {n} steps "
                         f"at {H}x{W} ({cs:.1f} s)"}
    if rank == 0:
        line = {
            "metric": "env-steps/sec, env step + render + frame stack only (SURVEY configs 1/3)",
            "value": world * B * args.steps / dt, "unit": "env-steps/s", "n_gpus": world, **dist_info(), "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: seeded resets, uniform random actions",
            "config": {"workload": f"{B} envs/GPU x {H}x{W} Breakout, {args.hist}-frame stack, no search",
                       "envs_per_gpu": B},
            "roofline": {"bound": "hbm", "kernel": "env_step_compact_kernel (step + render + history push)",
                         "achieved": achieved, "peak": 8000.0, "unit": "GB/s", "frac": achieved / 8000.0,
                         "traffic": traffic, "bytes_per_env_step": env_bytes(H, W), "avg_launch_ms": kms,
                         "kernel_timed": ktimed},
            "cpu_baseline": cpu,
        }
        check_fracs(line)
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def run_learner(args, world, rank, local):
    """RLSystem._training_stage minibatches (B windows, K = 5 unroll, train-mode
    BN, backward, Adam) on the device learner over a synthetic device replay ring. `value` =
    windows/s (all ranks; N > 1 = independent replicas, the reference's learner is single-device).
    roofline = the minibatch's algorithmic conv/linear FLOPs / its time vs the dense MFMA peak
    of the arithmetic type (f32 157.3 TF, bf16 2500 TF)."""
    from mzba.config import default_config
    from mzba.learner import Learner
    from mzba.weights import init_state_dict
    dt = args.dtype if args.dtype in ("f32", "bf16") else "f32"
    mcfg = default_config()["model"]
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    B, K, Lh, cap = args.minibatch, 5, mcfg["state_history_length"], 4096
    g = torch.Generator(device=dev).manual_seed(args.seed + rank)

    class Ring:
        pass
    ring = Ring()
    ring.start, ring.max_length, ring.length = 0, cap, cap
    ring._ring = {
        "states": (torch.randint(0, 8, (cap, Lh, 320), device=dev, generator=g) *
                   (torch.rand(cap, Lh, 320, device=dev, generator=g) < 0.3)).to(torch.uint8),
        "past_actions": torch.randint(0, 3, (cap, Lh), device=dev, generator=g),
        "future_actions": torch.randint(0, 3, (cap, K), device=dev, generator=g),
        "rewards": torch.randint(-1, 2, (cap, K), device=dev, generator=g).float(),
        "targets": torch.randn(cap, K, device=dev, generator=g) * 2,
        "counts": torch.randint(0, 51, (cap, K, 3), device=dev, generator=g).float() + 1,
    }
    ln = Learner(mcfg, init_state_dict(mcfg, args.seed), K=K, dtype=dt, device=dev, streams=args.learner_streams)
    slots = [torch.randperm(cap, device=dev, generator=g)[:B].to(torch.int32) for _ in range(args.warmup + args.steps)]
    for i in range(args.warmup):
        ln.train_minibatch(ring, slots[i])
    if not args.no_graph:  # the whole minibatch as one HIP graph (after an eager one: packs, scratch)
        if args.warmup == 0:
            ln.train_minibatch(ring, slots[0])
        ln.capture(ring, B)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(torch.cuda.current_stream())
        loss = ln.train_minibatch(ring, slots[args.warmup + i])
        ev[i][1].record(torch.cuda.current_stream())
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dtt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dtt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dtt = float(tt.item())
    kms = float(np.median([a.elapsed_time(c) for a, c in ev]))
    fl = ln.flops_per_minibatch(B)
    peak = 157.3 if dt == "f32" else PEAK_BF16_TFLOPS
    achieved = fl / (kms * 1e-3) / 1e12
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        from oracle.learner import LearnerOracle
        from mzba.learner import MinibatchRing  # noqa: F401
        nb = 8
        torch.set_num_threads(min(16, os.cpu_count() or 1))
        gen = np.random.default_rng(args.seed)
        lut = np.array([0, 0.3, 0.6, 1.0], np.float32)
        mb = dict(states=lut[gen.integers(0, 4, (nb, Lh, 16, 20)) * (gen.random((nb, Lh, 16, 20)) < 0.3)],
                  past_actions=gen.integers(0, 3, (nb, Lh)), future_actions=gen.integers(0, 3, (nb, K)),
                  rewards=gen.choice(np.array([-1, 0, 1], np.float32), (nb, K)),
                  targets=(gen.normal(size=(nb, K)) * 2).astype(np.float32),
                  counts=gen.multinomial(50, [0.3, 0.3, 0.4], (nb, K)).astype(np.float32) + 1)
        o = LearnerOracle(mcfg, init_state_dict(mcfg, args.seed), K=K)
        o.step(mb)
        c0, n = time.perf_counter(), 0
        while n < 3 and time.perf_counter() - c0 < 20.0:
            o.step(mb)
            n += 1
        cs = time.perf_counter() - c0
        cpu = {"value": nb * n / cs, "unit": "windows/s", "cores": torch.get_num_threads(), "kind": "port",
               "sample": f"oracle/learner.py (torch-CPU f32, the reference's ops) on {n} minibatches of {nb} "
                         f"windows ({cs:.1f} s)"}
    if rank == 0:
        line = {
            "metric": "learner windows/sec (RLSystem._training_stage minibatch: K=5 rollout, train-mode BN, "
                      "backward, Adam)",
            "value": world * B * args.steps / dtt, "unit": "windows/s", "n_gpus": world, **dist_info(), "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dtt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": dt,
            "data": "synthetic replay ring (4096 windows), seeded random-init reference-architecture nets",
            "config": {"workload": f"learner minibatch {B} windows x K=5, full-width nets (config.yaml)",
                       "minibatch": B, "parallelism": "replicas" if world > 1 else "single device"},
            "roofline": {"bound": "mfma", "kernel": "whole minibatch (conv fwd / dgrad / wgrad + BN + heads + Adam)",
                         "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
                         "traffic": None, "flop_per_minibatch": fl, "avg_launch_ms": kms,
                         # the minibatch's top kernels by kernel time (rocprof of this workload, with SQ figures of
                         # the two largest: profiles/learner_kernels.json), for the reader of the 0.2 above
                         "top_kernels": learner_kernels(B, dt)},
            "loss": float(loss[0]),
            "launch": "eager" if args.no_graph else "hip-graph replay of the whole minibatch",
            "streams": args.learner_streams,
            "cpu_baseline": cpu,
        }
        check_fracs(line)
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def big_conv_kernel(args, B, p):
    """The kernel the latent residual convs run on when the fused tower does not apply (config 3)."""
    from mzba import _lib as L
    if p.lh * p.lw <= 160:
        return "conv_lat"
    if args.dtype == "bf16" and not args.no_halo and L.lib().mzba_conv_halo_supported(p.lh, p.lw, p.c1, p.c1, 3):
        return "conv_halo"
    return "conv_big_bf16" if B * p.lh * p.lw >= 65536 and args.dtype == "bf16" else "conv_igemm"


def cfg_name(B, S, dyn=None):
    """Which BASELINE config an acting-loop run is (per-GPU batch, sims, dynamics precision)."""
    if (B, S) == (4096, 200):
        return "config 5" if dyn == "fp16" else "config 5 geometry (bf16 dynamics)"
    return {(1024, 50): "config 2",
            (4096, 50): "north_star (4096 envs x 50 sims on 1 MI355X; = config 4's per-GPU share)"}.get((B, S), "custom")


def step_flops(p, H, W, S):
    """Algorithmic FLOPs of one acting env-step: representation + root prediction +
    S x (dynamics + prediction), convs and linear heads, at this geometry (72.17 G at 16x20, S=50)."""
    c0, c1, hw = p.c0, p.c1, p.lh * p.lw
    fl, hh, ww, cin = 0.0, H, W, 2 * p.L
    for kind, layer in p.rep:
        if kind == "pool":
            hh, ww = hh // 2, ww // 2
            continue
        for c in ([layer] if kind == "conv" else list(layer)):
            ci = cin if c is p.rep[0][1] else c["cin"]
            fl += 2.0 * hh * ww * c["cout"] * c["ks"] ** 2 * ci
    conv = lambda ci, co, ks: 2.0 * hw * co * ks * ks * ci  # noqa: E731
    pred = 2 * len(p.pred) * conv(c1, c1, 3) + conv(c1, c1 // 2, 3) + conv(c1, c1 // 2, 1) + \
        2.0 * hw * (c1 // 2) * (3 + p.ns)
    dyn = conv(c1 + 3, c1, 3) + 2 * len(p.dyn) * conv(c1, c1, 3) + conv(c1, c1, 1) + 2.0 * hw * c1 * p.ns
    return fl + pred + S * (dyn + pred)


def tower_traffic(B, fused_tower, kname):
    """PMC HBM bytes per launch of the dominant kernel at this batch (profiles/tower_hbm_traffic.json,
    written by tools/pmc_summarize.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)."""
    tpath = os.path.join(ROOT, "profiles", "tower_hbm_traffic.json")
    if not (fused_tower and os.path.exists(tpath)):
        return None, None
    for rec in json.load(open(tpath))["records"]:
        if rec.get("envs") == B and rec.get("kernel_name") == kname:
            return rec.get("bytes_per_launch"), rec
    return None, None


def tower_counters(B, kname, sims, dyn):
    """Measured SQ counters of one template instance of the dominant kernel in the bench run with this batch,
    simulation count and dynamics precision (profiles/tower_sq_counters.json, from the two rocprofv3 --pmc passes
    of tools/gpu_run.sh 'sq' inside this bench): MFMA-pipe busy fraction of the SIMD cycles at the clock the
    chip held, LDS bank-conflict share, and the executed MFMA count. Keyed on the instance (towerp_kernel<1> is
    the fp16 dynamics step of config 5, towerp_kernel<0> every bf16 step), so a record is never quoted for
    launches it did not count."""
    tpath = os.path.join(ROOT, "profiles", "tower_sq_counters.json")
    if not os.path.exists(tpath):
        return None
    for rec in json.load(open(tpath))["records"]:
        if (rec.get("envs"), rec.get("kernel_name"), rec.get("sims", 50), rec.get("dyn_dtype")) == (B, kname, sims, dyn):
            return rec
    return None


def learner_kernels(B, dt):
    """The committed kernel breakdown of the learner minibatch (profiles/learner_kernels.json) when it was measured at
    this minibatch size and dtype, else None."""
    tpath = os.path.join(ROOT, "profiles", "learner_kernels.json")
    if not os.path.exists(tpath):
        return None
    rec = json.load(open(tpath))
    return rec if (rec.get("minibatch"), rec.get("dtype")) == (B, dt) else None


def conv_counters(B, H, W, kname):
    """PMC record of the non-fused path's dominant conv kernel (config 3's halo conv) at this batch and latent size
    (profiles/conv_counters.json, tools/gpu_run.sh step 'pmck' + tools/pmc_conv_summary.py: HBM bytes per launch from the
    FETCH_SIZE / WRITE_SIZE passes, MFMA busy / clock / LDS conflicts from the SQ passes of the same bench)."""
    tpath = os.path.join(ROOT, "profiles", "conv_counters.json")
    if not os.path.exists(tpath):
        return None
    for rec in json.load(open(tpath))["records"]:
        if (rec.get("envs"), rec.get("H"), rec.get("W")) == (B, H, W) and kname in rec.get("kernel_name", ""):
            return rec
    return None


def fp16_clock_note():
    """Config 5's fp16 dynamics net holds a lower clock than bf16 with the same instruction stream: register-only
    16x16x32 MFMA streams with random operands (profiles/mfma_clock_dtype.json, tools/mfma_clock_dtype.hip) run
    fp16 at ~0.94 of bf16's clock and ~0.96 of its rate — the fp16 multipliers' power, not this code."""
    tpath = os.path.join(ROOT, "profiles", "mfma_clock_dtype.json")
    if not os.path.exists(tpath):
        return None
    r = json.load(open(tpath))
    return {"bf16_core_ghz": r["bf16"]["core_ghz_median"], "fp16_core_ghz": r["fp16"]["core_ghz_median"],
            "fp16_over_bf16_clock": r["fp16_over_bf16_clock"], "fp16_over_bf16_rate": r["fp16_over_bf16_rate"],
            "cause": "fp16 MFMA streams hold a lower clock than bf16 under the power limit (register-only probe, "
                     "random operands): the fp16 step cannot match the bf16 one with the same instruction stream",
            "source": "profiles/mfma_clock_dtype.json"}


L2_PEAK_TBPS = 34.5  # MI355X L2 (8 XCDs x 4 MiB) aggregate read rate, MI355X_MICROARCH.md 'L2 (per XCD)'


def l2_weight_stream(conv_ms, C=256, n_cu=256):
    """The per-CU weight stream of a tower conv: every workgroup streams each conv's whole
    weight pack (C x 9C bf16 = 1.18 MB) from L2 into its registers whatever its env count, so a CU moves those
    bytes per conv. `frac` = that per-CU rate / the L2 peak per CU (34.5 TB/s / 256 CUs, the guide's chip figure).
    Beside it, not a bound: the rate tools/probes/l2_stream_probe.hip sustained with the tower's own access form
    (all 256 CUs streaming the 33 MB tower pack, profiles/l2_stream.json) — the kernel may exceed what that
    probe sustains, so it is reported as a ratio, never as a roofline fraction."""
    if not conv_ms:
        return None
    nbytes = C * 9 * C * 2
    rate = nbytes / (conv_ms * 1e-3) / 1e9
    peak = L2_PEAK_TBPS * 1e3 / n_cu
    out = {"bytes_per_cu_per_conv": nbytes, "measured_ms_per_conv": conv_ms, "achieved_per_cu_GBps": rate,
           "peak_per_cu_GBps": peak, "frac": rate / peak, "peak_source": "MI355X_MICROARCH.md L2 aggregate / 256 CUs"}
    tpath = os.path.join(ROOT, "profiles", "l2_stream.json")
    if os.path.exists(tpath):
        probe = json.load(open(tpath)).get("per_cu_GBps")
        if probe:
            out.update({"probe_per_cu_GBps": probe, "ratio_to_probe": rate / probe,
                        "probe_source": "profiles/l2_stream.json"})
    return out


# Fraction of a launch's algorithmic 3x3-conv FLOPs the kernel issues to the MFMA pipe: the reference's
# Conv2d(padding=1) on the 4x5 latent evaluates 50 of its 180 taps per env on zero padding. The pixel-tiled
# kernel (plan 4) skips them all (130 / 180); the column-tiled tower8 (plans 2 / 3) skips the dx ones only
# (39 of 45 tile-taps, 86.7 %).
EXECUTED_FRACTION = {"towerp_kernel<0>": 130.0 / 180.0, "towerp_kernel<1>": 130.0 / 180.0,
                     "tower8_kernel<0, 2>": 39.0 / 45.0, "tower8_kernel<0, 1>": 39.0 / 45.0}


def tower_kernel_name(B, fp16=False):
    """The kernel mzba_tower_plan picks for batch B (tower.hip), as rocprofv3 names the template instance
    (<1>: the fp16 element type of config 5's dynamics step)."""
    from mzba import _lib as L
    e = int(bool(fp16))
    return {2: f"tower8_kernel<{e}, 2>", 3: f"tower8_kernel<{e}, 1>", 4: f"towerp_kernel<{e}>"}.get(
        L.lib().mzba_tower_plan(B), f"tower_kernel<{e}>")


def x6_flops(p, H, W, S, x3=False):
    """Per env-step FLOPs of the f32 parity path's convs by the form they run in: split-fp16 x3 products (x3: the convs
    PackedNets gave 'wx3' — the 4x5 latent's towers, dynamics' first conv and heads' convs, and the representation's
    16x20 / 8x10 3x3 convs on the pre-split tiles), split-bf16 x6 products (conv_x6: the layers with 'wx' and no x3
    form in use) and the rest (f32-input MFMA convs and heads), at this geometry: (x3, x6, rest)."""
    conv = lambda c, hw: 2.0 * hw * c["cout"] * c["ks"] ** 2 * c["cin"]  # noqa: E731
    lat = {"x3": 0.0, "x6": 0.0}
    x6, hh, ww = 0.0, H, W
    for kind, layer in p.rep:
        if kind == "pool":
            hh, ww = hh // 2, ww // 2
            continue
        for c in ([layer] if kind == "conv" else list(layer)):
            if x3 and c.get("wx3") is not None:  # round 6: the representation's convs on the x3 pre-split tiles
                lat["x3"] += conv(c, hh * ww)
            elif c.get("wx") is not None:
                x6 += conv(c, hh * ww)
    hw = p.lh * p.lw

    def add(c, n):
        if x3 and c.get("wx3") is not None:
            lat["x3"] += n * conv(c, hw)
        elif c.get("wx") is not None:
            lat["x6"] += n * conv(c, hw)
    for c in [c for blk in p.pred for c in blk] + [p.pol_conv, p.val_conv]:
        add(c, 1 + S)
    for c in [c for blk in p.dyn for c in blk] + [p.dyn0, p.rew_conv]:
        add(c, S)
    x6 += lat["x6"]
    return lat["x3"], x6, step_flops(p, H, W, S) - x6 - lat["x3"]


X6_PEAK_TFLOPS = 2500.0 / 6  # six bf16 MFMAs per f32-faithful product
X3_PEAK_TFLOPS = 2500.0 / 3  # three fp16 MFMAs per split-fp16 product (fp16 dense MFMA = the bf16 rate)


def parity_roofline(p, H, W, S, ms_per_step, B, x3=False):
    """Roofline of the f32 parity path's step: its x3 convs against the dense fp16 peak / 3, its x6 convs against the
    dense bf16 peak / 6, the rest against the dense f32 MFMA peak; frac = the time all would take at their peaks / the
    measured time."""
    fx3, fx6, frest = x6_flops(p, H, W, S, x3)
    ideal_ms = B * (fx3 / (X3_PEAK_TFLOPS * 1e12) + fx6 / (X6_PEAK_TFLOPS * 1e12) + frest / (PEAK_F32_TFLOPS * 1e12)) * 1e3
    return {"flop_x3_per_env_step": fx3, "flop_x6_per_env_step": fx6, "flop_f32_per_env_step": frest,
            "peak_x3": X3_PEAK_TFLOPS, "peak_x6": X6_PEAK_TFLOPS,
            "peak_f32": PEAK_F32_TFLOPS, "peak": B * (fx3 + fx6 + frest) / (ideal_ms * 1e-3) / 1e12,
            "ideal_ms_per_step": ideal_ms, "frac": ideal_ms / ms_per_step}


def conv_flops(B, hw, C):
    return 2.0 * B * hw * C * 9 * C


PEAK_F32_TFLOPS = 157.3  # MI355X dense f32 MFMA (MI355X_MICROARCH.md chip table)


def want_parity(args, rank, world):
    return rank == 0 and world == 1 and not args.no_parity and args.dtype != "f32"


LOOP_STATE = ("paddle", "bx", "by", "dx", "dy", "done", "bricks", "cur_frame", "cur_src", "hist_frames", "hist_actions",
              "hist_len", "reward", "valid")


def snapshot_loop(loop):
    """Device copies of everything an acting step reads: the compact env state, the frame-history
    ring and the step context (search id, step index, record row)."""
    env = loop.env
    snap = {k: getattr(env, k).clone() for k in LOOP_STATE if getattr(env, k) is not None}
    snap["ctx"] = loop.ctx.clone()
    snap["ids"] = (loop.search_id, loop.step_index, loop.t)
    return snap


def restore_loop(loop, snap, B=None):
    """Restore a snapshot into `loop`; with B (the snapshot's batch) larger than the loop's, its first envs only (every
    env tensor is env-major, so a prefix of B_loop / B of it is the first envs' state)."""
    for k in LOOP_STATE:
        if k in snap:
            dst, src = getattr(loop.env, k), snap[k]
            if B is not None and src.shape[0] != dst.shape[0]:
                src = src.reshape(B, -1)[: loop.B].reshape(dst.shape)
            dst.copy_(src)
    loop.ctx.copy_(snap["ctx"])
    loop.search_id, loop.step_index, loop.t = snap["ids"]


def f32_parity_path(cfg, mcfg, sd, loop, snap, t0, args, B, H, W, nsub=None):
    """The first timed step replayed on the f32 parity path (networks within 1e-5 of the reference,
    bit-exact trees): the same env state, search id and keyed randomness as the benchmarked step. The parity
    path's 4x5-latent convs run as split-fp16 x3 products (round 6: three fp16 MFMAs per f32 product, about 22
    bits per operand), the representation's as split-bf16 x6 products; the same step is also replayed with the
    latent convs on x6 (round 5's parity path) and on the f32-input MFMA (conv_igemm, rounds 1-3) — the visit
    counts of all three must agree. Returns the fraction of the envs whose visit counts equal the benchmarked
    step's, the agreement of the parity forms, and their throughputs (second replays, HIP events) against their
    rooflines.
    nsub < B (config 3's 84x84 geometry, whose f32 node pool at 4096 envs would not fit beside the benchmarked
    loop's): the first nsub envs only, restored from the snapshot's env-major prefix; the same global env ids, so the
    same keyed noise and tie-breaks; the default form only (no A/B)."""
    from mzba.agent import MuZeroAgent
    from mzba.acting import ActingLoop
    nsub = nsub or B
    ag32 = MuZeroAgent(mcfg, dtype="f32", device=loop.agent.device)
    ag32.load_state_dict(sd)
    l32 = ActingLoop(cfg, ag32, nsub, seed=args.seed, env_offset=loop.env_offset, height=H, width=W,
                     n_envs_total=loop.n_envs_total, pow_threads=loop.pow_threads)
    l32.temperature = loop.temperature
    l32.search.noise_weight = loop.search.noise_weight
    l32.reset(0)
    fl = step_flops(ag32.packed, H, W, args.sims)
    p32 = ag32.packed
    has_x3 = p32.dyn0.get("wx3") is not None
    forms = [("x3", True, True)] if has_x3 else []
    forms += [("x6", True, False), ("f32mfma", False, False)] if nsub == B or not has_x3 else []
    forms = forms if nsub == B else forms[:1]
    runs = {}
    for name, x6, x3 in forms:
        for rn in (l32.ws.runner, l32.rep_runner):
            rn.use_x6, rn.use_x3 = x6, x3
        counts, ms = [], []
        for _ in range(2):  # the first replay also warms the path (scratch, code objects)
            restore_loop(l32, snap, B)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            l32.act(eager=True)
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
            counts.append(l32.rec["counts"][t0].cpu().numpy())
        runs[name] = (counts, ms, l32.rec["values"][t0].cpu().numpy())
    main = forms[0][0]
    counts, ms, v32 = runs[main]
    c16 = loop.rec["counts"][t0].cpu().numpy()[:nsub]
    same = (counts[-1] == c16).all(1)
    l1 = np.abs(counts[-1].astype(np.int64) - c16.astype(np.int64)).sum(1)
    v16 = loop.rec["values"][t0].cpu().numpy()[:nsub]
    eps = nsub / (ms[-1] * 1e-3)
    rl = parity_roofline(p32, H, W, args.sims, ms[-1], nsub, x3=main == "x3")

    def other(name):
        if name not in runs or name == main:
            return None
        cf, msf, vf = runs[name]
        eps_f = nsub / (msf[-1] * 1e-3)
        r = {"value": eps_f, "ms_per_step": msf[-1], "speedup": eps / eps_f,
             "visit_count_match": float((cf[-1] == counts[-1]).all(1).mean()),
             "value_max_abs_diff": float(np.abs(vf - v32).max()),
             "deterministic": bool((cf[0] == cf[1]).all())}
        r["frac"] = (eps_f * fl / 1e12 / PEAK_F32_TFLOPS if name == "f32mfma" else
                     parity_roofline(p32, H, W, args.sims, msf[-1], nsub)["frac"])
        return r
    out = {"match": float(same.mean()), "envs": nsub,
           "root_value_max_abs_diff": float(np.abs(v16 - v32).max()),
           # beside the exact-match fraction: how far the count rows are apart, and whether the most visited
           # action (what temperature sampling mostly picks at low T) agrees
           "l1_mean": float(l1.mean()), "l1_max": int(l1.max()),
           "top_action_agreement": float((counts[-1].argmax(1) == c16.argmax(1)).mean()),
           "path": {"dtype": ("f32 (4x5 latent convs as split-fp16 x3 products, representation convs as split-bf16 x6)"
                              if main == "x3" else "f32 (latent convs as split-bf16 x6 products)"),
                    "value": eps, "unit": "env-steps/s",
                    "ms_per_step": ms[-1], "achieved_tflops": eps * fl / 1e12,
                    # the x3 convs against 2500 / 3 TF, x6 against 2500 / 6 TF, the rest against 157.3 TF;
                    # `peak` = the blended ceiling
                    "peak": rl["peak"], "frac": rl["frac"], "roofline": rl,
                    "deterministic": bool((counts[0] == counts[1]).all()),
                    "value_max_abs_diff_where_counts_agree": float(np.abs(v16 - v32)[same].max()) if same.any() else None,
                    "envs": nsub, "form": main,
                    "vs_x6_path": other("x6"),
                    "vs_f32_mfma_path": other("f32mfma"),
                    "what": "one acting step of the same envs on the f32 parity path (separate launches per layer), "
                            "eager, HIP events around the step; vs_x6_path / vs_f32_mfma_path: the same with the "
                            "latent convs on the split-bf16 x6 form / the f32-input MFMA (visit_count_match: against "
                            "this path's counts)"}}
    del l32, ag32
    torch.cuda.empty_cache()
    return out


def launcher_argv(n, argv, port):
    """The child command `bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment) starts: one rank per GPU
    under torch.distributed.run on this node, rendezvous on 127.0.0.1, the same bench arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def world_from_env(gpus, env):
    """(world, rank, local) from the torchrun environment; refuses a world size that differs from --gpus, so a
    line can never report N GPUs while running another number of ranks."""
    world = int(env.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" in env and world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: the launcher and the flag disagree")
    return world, int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0"))


def dist_info():
    """What the collectives actually ran on: the ranks the process group holds and its backend ("nccl" is RCCL on
    ROCm; "gloo" only in the one-GPU rehearsal, MZBA_DIST_REHEARSAL=1)."""
    if dist.is_available() and dist.is_initialized():
        return {"ranks_seen": dist.get_world_size(), "backend": str(dist.get_backend()),
                "rehearsal": os.environ.get("MZBA_DIST_REHEARSAL") == "1"}
    return {"ranks_seen": 1, "backend": None, "rehearsal": False}


def self_launch(n):
    """`python bench.py --gpus N` without a torchrun environment: start the N ranks as a child process (before any
    GPU call in this process — no exec), let rank 0's JSON line through, exit with the child's return code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(launcher_argv(n, sys.argv[1:], port), env=env)


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args.gpus))
    world, rank, local = world_from_env(args.gpus, os.environ)
    if args.workload == "selfcheck":  # the launcher and process group alone (gloo, no GPU call): CPU tests
        if world > 1:
            dist.init_process_group("gloo")
        if rank == 0:
            print(json.dumps({"workload": "selfcheck", "n_gpus": world, **dist_info()}))
        if world > 1:
            dist.destroy_process_group()
        return
    if world > 1:
        # production: one rank per GPU over RCCL. Rehearsal on a one-GPU box (MZBA_DIST_REHEARSAL=1):
        # every rank on cuda:0, gloo collectives — the same code path minus RCCL itself
        if os.environ.get("MZBA_DIST_REHEARSAL") == "1":
            local = 0
            torch.cuda.set_device(0)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if args.workload == "env":
        return run_env(args, world, rank, local)
    if args.workload == "learner":
        return run_learner(args, world, rank, local)
    from mzba.config import default_config
    from mzba.weights import init_state_dict
    from mzba.agent import MuZeroAgent
    from mzba.acting import ActingLoop
    from mzba.shard import TrajectoryGather
    from mzba import _lib as L

    if args.tower_variant:
        L.call("mzba_tower_set_variant", args.tower_variant)
    if args.halo_form is not None:
        L.call("mzba_conv_halo_set_form", args.halo_form)
    cfg = default_config()
    cfg["num_simulations"] = args.sims
    mcfg = cfg["model"]
    B = args.envs
    # frame geometry: 16x20 / 32-frame stack (the reference's), or --height/--width/--hist for
    # config 3's acting geometry (84x84, 4-frame stack, latent 21x21 after the two pools)
    H, W = args.height or 16, args.width or 20
    custom_geom = (H, W) != (16, 20)
    if custom_geom:
        mcfg["state_history_length"] = args.hist
        mcfg["latent_resolution"] = [H // 4, W // 4]
    agent = MuZeroAgent(mcfg, dtype=args.dtype, device=f"cuda:{local}", dyn_dtype=args.dyn_dtype)
    if world > 1:  # rank 0 holds the (learner's) weights; the target-net refresh hands them out
        from mzba.shard import broadcast_state_dict
        sd = broadcast_state_dict(mcfg, init_state_dict(mcfg, args.seed) if rank == 0 else None, agent.device)
        sd = {k: v.numpy() for k, v in sd.items()}
    else:
        sd = init_state_dict(mcfg, args.seed)
    agent.load_state_dict(sd)
    loop = ActingLoop(cfg, agent, B, seed=args.seed, env_offset=rank * B, height=H, width=W, n_envs_total=world * B,
                      pow_threads=args.pow_threads)
    if args.no_halo:
        loop.ws.runner.use_halo = False
        loop.rep_runner.use_halo = False
    gather = TrajectoryGather(world, rank, RECORD_K, B, H * W, f"cuda:{local}")
    loop.reset(0)
    last_flush = [0]

    def one_step(eager=False):
        if loop.t >= loop.max_steps or (loop.t > 0 and loop.all_done()):
            flush()
            gather.fence()  # the new episode rewrites record row 0..: after the last pack
            loop.reset()
            last_flush[0] = 0
        loop.act(eager=eager)
        if loop.t - last_flush[0] >= RECORD_K:
            flush()

    def flush():
        if loop.t > last_flush[0]:
            gather.exchange(loop.rec, last_flush[0], loop.t)
            last_flush[0] = loop.t

    for _ in range(args.warmup):
        one_step(eager=True)
    if not args.no_graph:
        loop.capture()  # one acting step (~S x 65 launches) as a HIP graph, replayed per step

    # ---- visit-count match + CPU baseline on a bounded sample (rank 0, N=1 only) -------
    cpu_info, match, match_f32 = None, None, None
    want_cpu = rank == 0 and world == 1 and not args.no_cpu and not custom_geom
    if want_cpu:
        nb = min(args.cpu_envs, B)
        cs = loop.cs
        x32 = torch.empty(B * 320 * cs, dtype=torch.float32, device=agent.device)
        loop.env.build_rep_input(x32, cs, False)
        sid = loop.search_id
        t_before = loop.t
        one_step()
        torch.cuda.synchronize()
        gpu_counts = loop.rec["counts"][t_before].cpu().numpy()[:nb] if loop.t == t_before + 1 else None
        noise = loop.ws.tree.noise.cpu().numpy()[:nb]
        x = x32.view(B, 16, 20, cs)[:nb, :, :, : 2 * loop.Lh].permute(0, 3, 1, 2).cpu().numpy()
        # the reference's CPU structure: torch-CPU f32 nets (the reference's own ops,
        # eval-mode BN) batched over the envs, per-env dict trees walked serially in Python
        from oracle.mcts import MCTSOracle
        from oracle.nets_torch import TorchNetModel
        torch.set_num_threads(min(16, os.cpu_count() or 1))
        nthreads = torch.get_num_threads()
        model = TorchNetModel(sd, mcfg)
        t0 = time.perf_counter()
        h = model.representation(np.ascontiguousarray(x)).numpy()
        _, oc = MCTSOracle(cfg, model, args.seed).search(h, noise, sid)
        cpu_s = time.perf_counter() - t0
        if gpu_counts is not None:
            match = float((gpu_counts == oc).all(1).mean())
        # the same envs through the f32 parity path of this build (same keyed noise / tie-breaks)
        from mzba.search import MCTSSearchVec
        agent32 = MuZeroAgent(mcfg, dtype="f32", device=agent.device)
        agent32.load_state_dict(sd)
        h32 = agent32.create_hidden_state_root(torch.from_numpy(np.ascontiguousarray(x)).to(agent.device))
        s32 = MCTSSearchVec(cfg, agent32, None, seed=args.seed, env_offset=0)
        s32.search_id = sid
        _, c32 = s32.search(h32)
        match_f32 = float((c32.numpy() == oc).all(1).mean())
        cpu_info = {"value": nb / cpu_s, "unit": "env-steps/s", "cores": nthreads, "kind": "port",
                    "sample": f"oracle port of the reference acting step (torch-CPU f32 nets = the reference's ops, "
                              f"per-env Python trees): representation + {args.sims}-sim search for {nb} envs of the "
                              f"bench's own state, 1 acting step ({cpu_s:.1f} s)"}

    # the state before the first timed step: the f32 parity path replays that step afterwards
    snap = snapshot_loop(loop) if want_parity(args, rank, world) else None
    t_snap = loop.t

    # ---- timed region ---------------------------------------------------------------------
    probe = []
    runner = loop.ws.runner
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        # the middle step runs eagerly with HIP events around every latent residual conv
        # (the dominant kernel) to measure its launch duration live inside the timed region
        probe_step = i == args.steps // 2
        runner.probe = probe if probe_step else None
        one_step(eager=probe_step)
    flush()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    runner.probe = None
    if world > 1:
        tt = torch.tensor([dt], device=agent.device, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    value = world * B * args.steps / dt
    runner.probe_collect()  # probe entries: (ms, convs in the launch), HIP events on the launch stream
    # per-conv average over the latent residual convs
    conv_ms = (float(sum(ms for ms, _ in probe) / sum(n for _, n in probe))) if probe else None
    tower_launch_ms = (float(np.mean([ms for ms, n in probe if n > 1])) if any(n > 1 for _, n in probe) else None)
    parity = None
    if snap is not None:  # after the timed region: nothing here is timed in `value`
        parity = f32_parity_path(cfg, mcfg, sd, loop, snap, t_snap, args, B, H, W,
                                 nsub=min(B, args.parity_envs) if custom_geom else None)
    p = agent.packed
    fl = conv_flops(B, p.lh * p.lw, p.c1)
    achieved = fl / (conv_ms * 1e-3) / 1e12 if conv_ms else None
    kname = tower_kernel_name(B) if tower_launch_ms else None
    traffic, traffic_rec = tower_traffic(B, any(n > 1 for _, n in probe), kname)
    ex_frac = EXECUTED_FRACTION.get(kname)
    sq = tower_counters(B, kname, args.sims, args.dyn_dtype) if kname else None
    # config 5: the fp16 dynamics step is its own instance (towerp_kernel<1>), counted separately
    kname16 = tower_kernel_name(B, fp16=True) if (kname and args.dyn_dtype == "fp16") else None
    sq16 = tower_counters(B, kname16, args.sims, args.dyn_dtype) if kname16 else None
    if not tower_launch_ms:  # config 3: the per-conv kernel's own PMC record (traffic and SQ figures)
        crec = conv_counters(B, p.lh, p.lw, big_conv_kernel(args, B, p) + "_kernel")
        if crec:
            traffic, sq = crec.get("bytes_per_launch"), crec
            traffic_rec = {"algorithmic_bytes": crec.get("algorithmic_bytes"), "source": "profiles/conv_counters.json"}
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            **dist_info(),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype + ("; dynamics fp16" if args.dyn_dtype == "fp16" else ""),
            "data": "synthetic: seeded random-init reference-architecture nets, seeded Breakout episodes",
            "config": {"workload": (f"{cfg_name(B, args.sims, args.dyn_dtype)}: {B} envs/GPU x {args.sims} MCTS sims, "
                                    "16x20 Breakout, 32-frame stack") if not custom_geom else
                                   (f"config 3 acting geometry: {B} envs/GPU x {args.sims} MCTS sims, {H}x{W} Breakout, "
                                    f"{args.hist}-frame stack, latent {H // 4}x{W // 4} (generic conv kernels)"),
                       "envs_per_gpu": B, "global_envs": world * B, "sims": args.sims,
                       "pow_threads": args.pow_threads,
                       "parallelism": f"env-sharded x{world}, RCCL gather of trajectory records to rank 0, target-net broadcast"},
            "roofline": {"bound": "mfma",
                         "kernel": (f"{kname} (fused dynamics / prediction step: 14-block residual "
                                    "tower, bf16 3x3 256->256 convs, M=B*20, N=256, K=2304 each)"
                                    + (f"; the dynamics step on {kname16} (fp16)" if kname16 else ""))
                                   if tower_launch_ms else
                                   (f"latent residual conv bf16 3x3 256->256 (M=B*{p.lh * p.lw},N=256,K=2304; "
                                    f"{big_conv_kernel(args, B, p)} kernel)"),
                         "achieved": achieved, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": (achieved / PEAK_BF16_TFLOPS) if achieved else None, "traffic": traffic,
                         "traffic_algorithmic_bytes": traffic_rec and traffic_rec.get("algorithmic_bytes"),
                         # the floor with per-XCD L2s: every one of the 8 XCDs fetches the tower's weights
                         # once (33 MB each), the latents once in all
                         "traffic_per_xcd_floor_bytes": traffic_rec and tower_launch_ms and (
                             traffic_rec.get("algorithmic_bytes") + 7 * (2 * 14 * 256 * 2304 * 2)),
                         "traffic_source": traffic_rec and traffic_rec.get("source", "profiles/tower_hbm_traffic.json"),
                         "flop_per_conv": fl, "avg_ms_per_conv": conv_ms, "avg_launch_ms": tower_launch_ms or conv_ms,
                         "launches_timed": len(probe),
                         # what the MFMA pipe actually issues: the algorithmic rate x the kernel's padding-free
                         # fraction of the 3x3 taps, against the same dense peak (live, this run)
                         "executed_fraction_of_algorithmic": ex_frac,
                         "executed_frac": (achieved * ex_frac / PEAK_BF16_TFLOPS) if (achieved and ex_frac) else None,
                         # measured PMC of the same kernel in this bench (profiled run, not this one)
                         "mfma_busy": sq and sq.get("mfma_busy"),
                         "mfma_busy_clock_ghz": sq and sq.get("clock_ghz"),
                         "lds_bank_conflict_frac": sq and sq.get("lds_bank_conflict_frac"),
                         "counters_source": sq and sq.get("source"),
                         "counters_kernel": sq and sq.get("kernel_name"),
                         # config 5: the fp16 dynamics instance's own counters (not the bf16 record reused)
                         "counters_dynamics_fp16": sq16 and {k: sq16.get(k) for k in (
                             "kernel_name", "mfma_busy", "clock_ghz", "wait_inst", "duration_ns",
                             "lds_bank_conflict_frac", "source")},
                         # below 16 x CUs envs a CU holds too few envs to hide its weight stream: the bound there
                         "l2_weight_stream": l2_weight_stream(conv_ms) if tower_launch_ms else None,
                         # config 5: why the fp16 dynamics step runs slower than bf16 (a property of the fp16 MFMA)
                         "fp16_clock": fp16_clock_note() if args.dyn_dtype == "fp16" else None},
            "cpu_baseline": cpu_info,
            "visit_count_match": match,
            "visit_count_match_sample": (f"{min(args.cpu_envs, B)} envs, bf16 HIP path vs the f32 CPU port (same keyed "
                                         "noise / tie-breaks)") if match is not None else None,
            "visit_count_match_f32_path": match_f32,
            # every env of the first timed step: the benchmarked bf16 path against this build's f32
            # parity path (1e-5 nets, bit-exact trees) replaying that step from the same state
            "visit_count_match_full": parity and parity["match"],
            "visit_count_l1_full": parity and {"mean": parity["l1_mean"], "max": parity["l1_max"], "sims": args.sims},
            "top_action_agreement_full": parity and parity["top_action_agreement"],
            "visit_count_match_full_sample": parity and (
                (f"all {B} envs" if parity["envs"] == B else f"the first {parity['envs']} of the {B} envs") +
                f" of the first timed step: {args.dtype} HIP path vs the f32 HIP parity path from the "
                "same env state, search id and keyed noise / tie-breaks"),
            "root_value_max_abs_diff_full": parity and parity["root_value_max_abs_diff"],
            "parity_path": parity and parity["path"],
            "launch": "eager" if args.no_graph else "hip-graph replay (probe step eager)",
            "whole_step_mfma_frac": (B * world * step_flops(agent.packed, H, W, args.sims) * args.steps / dt / 1e12)
                                    / (PEAK_BF16_TFLOPS * world),
            "flop_per_env_step": step_flops(agent.packed, H, W, args.sims),
        }
        check_fracs(out)
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def check_fracs(out, path="bench"):
    """Every roofline fraction in the line is measured against a true ceiling, so none may exceed 1: a value above
    it means a wrong denominator, and the bench fails instead of printing it."""
    if isinstance(out, dict):
        for k, v in out.items():
            if (k == "frac" or k.endswith("_frac")) and isinstance(v, (int, float)) and v > 1.0:
                raise SystemExit(f"bench.py: {path}.{k} = {v:.4f} > 1 — a fraction of a peak above the peak is a "
                                 "wrong denominator, not a result")
            check_fracs(v, f"{path}.{k}")


if __name__ == "__main__":
    main()
