#!/usr/bin/env python
"""Throughput of AutoEncoderRGB_Journal encode+decode on MI355X (BASELINE.json metric).

One "step" = one full forward (encoder, hyperprior, 10-slice entropy model,
decoder, bpp + masked MSE) of a synthetic 256x256 RGBA batch of 8 per GPU
(BASELINE config 2), inputs resident in HBM, replayed from a HIP graph.
N > 1: one process per GPU (torchrun), independent replicas (inference has no
exchange step), barrier + synchronize around the timed region, MAX over ranks.

Rank 0 also prints, in the same JSON line:
  roofline      -- the dominant kernel's algorithmic FLOP/s (HIP events on the
                   launching stream, eager attribution pass) vs its peak;
  cpu_baseline  -- the CPU oracle (fp32 PyTorch restatement of the reference)
                   on a bounded sample of the same workload, on this host.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "deep-learning-based-rgba-image-compression-with-masked-window-based-attention_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "MPixels/sec encode+decode, 256×256 RGBA batch; bpp & PSNR parity vs reference"
TRAIN_METRIC = "MPixels/sec training step (fwd+bwd+clamp+Adam), 256×256 RGBA batch"
PEAK = {"bf16": {"mfma": 2500.0, "hbm": 8000.0}, "f32": {"mfma": 157.3, "hbm": 8000.0}}


def synth_inputs(B, H, W, seed=0):
    """RGB k/255; alpha cycles ones / left-half-zero / ellipse with an
    8-px linear ramp (k/255) / zero; masked_input = where(alpha > 0, rgb, alpha)."""
    g = torch.Generator().manual_seed(seed)
    rgb = torch.round(torch.rand((B, 3, H, W), generator=g) * 255) / 255
    a = torch.ones((B, 1, H, W))
    yy, xx = torch.meshgrid(torch.arange(H).float(), torch.arange(W).float(), indexing="ij")
    for b in range(B):
        k = b % 4
        if k == 1:
            a[b, :, :, : W // 2] = 0
        elif k == 2:
            r = (((yy - H / 2) / (0.35 * H)) ** 2 + ((xx - W / 2) / (0.45 * W)) ** 2).sqrt()
            ramp = torch.clamp((1.0 - r) * (0.4 * min(H, W)) / 8.0, 0, 1)
            a[b, 0] = torch.round(ramp * 255) / 255
        elif k == 3:
            a[b].zero_()
    return torch.where(a > 0, rgb, a), a


# Attribution runs enqueue one eager step behind a GPU spin (torch.cuda._sleep, in clock
# cycles) long enough for the host to queue every launch first, so the per-launch HIP-event
# intervals measure back-to-back GPU execution as in the graph replay, not host launch gaps.
SPIN_FWD = 150_000_000
SPIN_TRAIN = 600_000_000


LATENT_GAIN = 20.0     # tests/golden/make_golden.py: Encoder.x4 scaled so symbols are non-zero


def rgb_net(latent_gain=LATENT_GAIN):
    """Seed-234 random-init AutoEncoderRGB_Journal with Encoder.x4 (1x1 192 -> 80, the conv
    feeding the latent) scaled by ``latent_gain``: at plain random init every latent symbol
    round(y - mu) is 0 and bpp parity would be vacuous; with 20 they span about -5..10 like a
    trained codec's.  Same architecture and FLOPs."""
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    torch.manual_seed(234)
    net = AutoEncoder().eval()
    with torch.no_grad():
        net.Encoder.x4.weight.mul_(latent_gain)
        net.Encoder.x4.bias.mul_(latent_gain)
    return net


def mask_net(latent_gain=LATENT_GAIN):
    """Seed-234 random-init AutoEncoderMask_Journal with EncoderMask.7 (1x1 192 -> 80, the conv
    feeding the last attention block and the latent) scaled by ``latent_gain``, for the same
    reason as rgb_net: non-zero latent symbols."""
    from rgbac.models.AutoEncoderMask_Journal import AutoEncoder
    torch.manual_seed(234)
    net = AutoEncoder().eval()
    with torch.no_grad():
        net.EncoderMask[7].weight.mul_(latent_gain)
        net.EncoderMask[7].bias.mul_(latent_gain)
    return net


def host_cores():
    """CPU cores this process may run on (len(os.sched_getaffinity(0)))."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _set_cpu_threads():
    """torch threads for the CPU baseline = len(sched_getaffinity(0)), capped by
    OMP_NUM_THREADS when the job's CPU share sets it (the GPU box: 16) -- more threads than
    the share oversubscribes it.  Returns the thread count actually used."""
    n = host_cores()
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    torch.set_num_threads(n)
    return n


def parity_sample(S=256, n=4):
    """The parity / CPU-baseline sample: the first ``n`` images of the bench batch (one per
    alpha pattern: ones, left-half zero, ramped ellipse, all zero), seed 0."""
    x, a = synth_inputs(n, S, S, seed=0)
    return x, a


def cpu_baseline(budget_s, S=256):
    """Oracle (CPU fp32 restatement of the reference) on the 4-image parity sample (one image
    per forward, B=1, as trainRGB.py's Kodak loop runs), this host's cores, cycling over the
    sample until ``budget_s``.  Returns (baseline record, oracle outputs of the first pass:
    [(bpp, mse, MS-SSIM of the clamped x_hat)] per image) -- the outputs are the parity reference of the
    bench line (the oracle is used here only as the checker / timed CPU baseline)."""
    from oracle import ref_metrics
    from oracle import ref_model as ref
    cores = _set_cpu_threads()
    sd = {k: v.detach().cpu() for k, v in rgb_net().state_dict().items()}
    x, a = parity_sample(S)
    outs = []
    with torch.no_grad():
        mes = [ref.supply_mask(a[i:i + 1]) for i in range(x.shape[0])]
        for i in range(x.shape[0]):                    # first pass = warm-up + parity outputs
            o = ref.rgb_forward(sd, x[i:i + 1], a[i:i + 1], a[i:i + 1], *mes[i][:4])
            msv = ref_metrics.ms_ssim(x[i:i + 1], o[0].clamp(0, 1), data_range=1.0).item()
            outs.append((o[2].item(), o[1].item(), msv))
        n, t0 = 0, time.perf_counter()
        while True:
            i = n % x.shape[0]
            ref.rgb_forward(sd, x[i:i + 1], a[i:i + 1], a[i:i + 1], *mes[i][:4])
            n += 1
            if (time.perf_counter() - t0 >= budget_s and n >= x.shape[0]) or n >= 4000:
                break
        dt = time.perf_counter() - t0
    rec = {"value": round(n * S * S / dt / 1e6, 4), "unit": "MPix/s", "cores": cores,
           "kind": "port",
           "sample": f"oracle rgb_forward fp32 on the 4-image parity sample ({S}x{S}, B=1 per "
                     f"forward, alpha ones/half/ellipse/zero), {n} timed forwards after 1 "
                     f"warm-up pass, {dt:.1f} s, torch threads {cores} (sched_getaffinity {host_cores()})"}
    return rec, outs


def gpu_parity(net, dev, outs_ref, S=256, account=False):
    """bpp / PSNR / MS-SSIM of the HIP forward (net's current compute dtype) on the parity
    sample, one image per forward, against the oracle's outputs ``outs_ref``
    (trainRGB.py:289-311: PSNR from the model's masked MSE, MS-SSIM of the clamped x_hat).
    ``account`` (fp32 mode): per image, every latent symbol round(y - mu) compared with the
    teacher-forced oracle (oracle/parity.py): flips, how many sit at near-ties, and the
    teacher-forced PSNR / MS-SSIM / bpp deltas (outside the timed region, checker only)."""
    import math
    from rgbac.layers.SupplyMask import mask_pyramid
    from rgbac.metrics.ms_ssim_torch import ms_ssim
    from rgbac.models._latent import debug_views
    x, a = parity_sample(S)
    d_bpp = d_psnr = d_ms = 0.0
    rel_bpp = 0.0
    per = []
    acc = {"flips": 0, "near_tie_flips": 0, "far_flips": 0, "z_flips": 0, "z_far_flips": 0,
           "symbols": 0, "nonzero_symbols": 0, "noise_floor": 0.0, "tf_max_abs_d_psnr_db": 0.0,
           "tf_max_abs_d_ms_ssim": 0.0, "max_bits_unflipped_rel": 0.0}
    sd = None
    if account:
        from oracle import parity
        sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    from rgbac import runtime as rt
    for i in range(x.shape[0]):
        xi, ai = x[i:i + 1].to(dev), a[i:i + 1].to(dev)
        _, me = mask_pyramid(ai, 4)
        dbg = {} if account else None
        with torch.no_grad(), rt.fixed_tiles():        # shape-rule tiles: no autotune pass
            o = net(xi, ai, ai, *me, debug=dbg)
        bpp, mse = o[2].item(), o[1].item()
        rec_acc = None
        if account:
            rep = parity.north_star_report(sd, "rgb", x[i:i + 1], a[i:i + 1], debug_views(dbg),
                                           (o[0].cpu(), mse, bpp))
            for k in ("flips", "near_tie_flips", "far_flips", "z_flips", "z_far_flips",
                      "symbols", "nonzero_symbols"):
                acc[k] += rep.get(k, 0)
            acc["noise_floor"] = max(acc["noise_floor"], rep["noise_floor"])
            acc["tf_max_abs_d_psnr_db"] = max(acc["tf_max_abs_d_psnr_db"], rep["tf_d_psnr_db"] or 0.0)
            acc["tf_max_abs_d_ms_ssim"] = max(acc["tf_max_abs_d_ms_ssim"], rep["tf_d_ms_ssim"] or 0.0)
            acc["max_bits_unflipped_rel"] = max(acc["max_bits_unflipped_rel"],
                                                rep["bits_unflipped_rel"])
            rec_acc = {"flips": rep["flips"], "near_tie_flips": rep["near_tie_flips"],
                       "far_flips": rep["far_flips"], "z_flips": rep.get("z_flips", 0),
                       "per_slice_flips": rep["per_slice_flips"],
                       "tf_d_psnr_db": None if rep["tf_d_psnr_db"] is None
                       else float(f"{rep['tf_d_psnr_db']:.3g}"),
                       "tf_d_ms_ssim": None if rep["tf_d_ms_ssim"] is None
                       else float(f"{rep['tf_d_ms_ssim']:.3g}")}
        rb, rm, rms = outs_ref[i]
        psnr = 10 * math.log10(1.0 / mse) if mse > 0 else None
        rpsnr = 10 * math.log10(1.0 / rm) if rm > 0 else None
        msv = ms_ssim(xi, o[0].clamp(0, 1), data_range=1.0).item()
        d_bpp = max(d_bpp, abs(bpp - rb))
        rel_bpp = max(rel_bpp, abs(bpp - rb) / max(abs(rb), 1e-12))
        if psnr is not None and rpsnr is not None:
            d_psnr = max(d_psnr, abs(psnr - rpsnr))
        d_ms = max(d_ms, abs(msv - rms))
        per.append({"bpp": round(bpp, 6), "bpp_ref": round(rb, 6),
                    "psnr": None if psnr is None else round(psnr, 4),
                    "psnr_ref": None if rpsnr is None else round(rpsnr, 4),
                    "ms_ssim": round(msv, 6), "ms_ssim_ref": round(rms, 6)})
        if rec_acc is not None:
            per[-1]["symbols"] = rec_acc
    res = {"max_abs_d_bpp": float(f"{d_bpp:.3g}"), "max_rel_d_bpp": float(f"{rel_bpp:.3g}"),
           "max_abs_d_psnr_db": float(f"{d_psnr:.3g}"), "max_abs_d_ms_ssim": float(f"{d_ms:.3g}"),
           "per_image": per}
    if account:
        acc = {k: (float(f"{v:.3g}") if isinstance(v, float) else v) for k, v in acc.items()}
        acc["bar"] = ("integer symbols: every flip at a near-tie (far_flips == 0); teacher-forced "
                      "(oracle fed the device y_hat / z_hat) |dPSNR| < 1e-4 dB, |dMS-SSIM| < 1e-4; "
                      "bits over unflipped symbols equal")
        acc["bar_met"] = bool(acc["far_flips"] == 0 and acc["z_far_flips"] == 0 and
                              acc["tf_max_abs_d_psnr_db"] < 1e-4 and
                              acc["tf_max_abs_d_ms_ssim"] < 1e-4)
        res["symbol_accounting"] = acc
    return res


def cpu_baseline_train(budget_s):
    """Oracle training step (fp32 autograd on CPU: forward + backward of
    4096*mse + bpp) on 1 image of the same workload, this host's cores."""
    from oracle import ref_model as ref
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    cores = _set_cpu_threads()
    torch.manual_seed(234)
    sd = {k: v.detach().cpu().clone().requires_grad_(v.is_floating_point())
          for k, v in AutoEncoder().train().state_dict().items()}
    x, a = synth_inputs(2, 256, 256, seed=0)
    x, a = x[1:2], a[1:2]
    me = ref.supply_mask(a)
    g = torch.Generator().manual_seed(1)

    def one():
        nz = torch.rand((1, 192, 4, 4), generator=g) - 0.5
        ny = torch.rand((1, 80, 32, 32), generator=g) - 0.5
        out = ref.rgb_forward(sd, x, a, a, *me[:4], training=True, noise_z=nz, noise_y=ny)
        (4096 * out[1] + out[2]).backward()
    one()
    n, t0 = 0, time.perf_counter()
    while True:
        one()
        n += 1
        if time.perf_counter() - t0 >= budget_s or n >= 1000:
            break
    dt = time.perf_counter() - t0
    return {"value": round(n * 256 * 256 / dt / 1e6, 4), "unit": "MPix/s",
            "cores": cores, "kind": "port",
            "sample": f"oracle rgb_forward(training) + autograd backward fp32, 1 image 256x256 "
                      f"(half-transparent alpha), {n} timed iterations after 1 warm-up, {dt:.1f} s"}


def latest_profile(suffix):
    """profiles/rNN_<suffix> of the latest round that has one (or None)."""
    import glob
    hits = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_{suffix}")))
    return hits[-1] if hits else None


def pmc_traffic(kernel, path, config=None):
    """HBM bytes per dispatch of ``kernel`` from a committed rocprofv3 PMC summary
    (tools/profile_round.sh + tools/pmc_traffic.py: FETCH_SIZE x2 + WRITE_SIZE) taken on the
    same workload (``config``: batch / size / dtype), or None."""
    if not path or not os.path.exists(path):
        return None
    with open(path) as fh:
        d = json.load(fh)
    if config is not None and d.get("config") not in (None, config):
        return None
    ent = d.get("kernels", {}).get(kernel)
    return None if ent is None else ent["hbm_bytes_per_dispatch"]


def tune_cache_setup(args, default):
    """Load the committed per-shape tile choices (so the timed run and a rocprofv3 trace of
    it contain no autotuning dispatches); --save-tune writes the cache after warm-up."""
    from rgbac import runtime as rt
    path = args.tune_cache if args.tune_cache is not None else default
    if path and os.path.exists(path):
        rt.load_tune_cache(path)
        return path
    return None


def roofline_of(summ, dtype, nrep, traffic_file=None, config=None):
    total_ms = sum(d["ms"] for d in summ.values())
    dom_name, dom = max(summ.items(), key=lambda kv: kv[1]["ms"])
    per_ms = dom["ms"] / dom["launches"]
    per_fl = dom["flops"] / dom["launches"]
    achieved = per_fl / (per_ms * 1e-3) / 1e12
    peak = PEAK[dtype]["mfma"]
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            "traffic": pmc_traffic(dom_name, traffic_file, config),
            "kernel": dom_name,
            "avg_launch_us": round(per_ms * 1e3, 2),
            "algorithmic_gflop_per_launch": round(per_fl / 1e9, 4),
            "share_of_step": round(dom["ms"] / total_ms, 3)}, total_ms


def write_layers(prof, path, nrep):
    lay = prof.layers()
    tot = sum(v[1] for v in lay.values())
    with open(path, "w") as fh:
        for k, v in sorted(lay.items(), key=lambda kv: -kv[1][1]):
            fh.write(f"{v[1] / nrep:9.4f} ms {100 * v[1] / tot:5.1f}% n={v[0] // nrep:3d} "
                     f"{v[2] / max(v[1], 1e-9) / 1e9:8.1f} TF/s  "
                     f"{v[3] / max(v[1], 1e-9) / 1e6:7.0f} GB/s  {k}\n")


def main_train(args, world, rank, dev, dist):
    """BASELINE config 3 (1 GPU, batch 16) / config 5 (torchrun, 16 per GPU, RCCL)."""
    from rgbac import runtime as rt
    from rgbac.layers.SupplyMask import mask_pyramid
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    from rgbac.optim import AdamClamp
    from rgbac.parallel import DataParallelTrainer

    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    torch.manual_seed(234)
    net = AutoEncoder().train().to(dev).set_compute_dtype(dt)
    opt = AdamClamp(net.parameters(), lr=1e-4, clip=5.0)
    trainer = DataParallelTrainer(net, opt)
    B, S = args.batch, args.size
    x, a = synth_inputs(B, S, S, seed=rank)
    x, a = x.to(dev), a.to(dev)
    _, me = mask_pyramid(a, 4)

    def step():
        out = net(x, a, a, *me)
        loss = 4096.0 * out[1] + out[2]                 # trainRGB.py:183-198 (lambda 4096)
        trainer.step(loss)
        # only the detached loss leaves the step: a live output would keep this step's
        # autograd graph -- and its AccumulateGrad nodes, bound to the stream they were
        # created on -- alive into the next (captured) step
        return loss.detach()

    tuned = tune_cache_setup(args, os.path.join(ROOT, "profiles", f"tune_train_{args.dtype}_b{B}_{S}.json"))
    step()                    # tunes; with DP buckets this is also their learning step
    torch.cuda.synchronize()
    if args.save_tune and rank == 0:
        rt.save_tune_cache(args.save_tune)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # The whole step -- forward, backward (with the bucketed RCCL all-reduces under DP),
    # clamp + Adam (device step counter) -- is captured once and replayed from a HIP graph at
    # every world size, so the host's per-launch cost leaves the timed loop.
    run, graph, gout = capture_train(step, opt, dev, args.no_graph)
    captured = graph is not None
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = run()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ms = elapsed / args.steps * 1e3
    value = world * B * S * S * args.steps / elapsed / 1e6
    loss_val = out.item()
    del out, run
    if graph is not None:
        del gout, graph                       # the captured graph's autograd nodes
    if rank == 0:
        prof = rt.LaunchProfiler()
        rt.PROFILER = prof
        for _ in range(2):
            torch.cuda._sleep(SPIN_TRAIN)   # queue the whole step behind a spin: GPU-side times
            step()
        rt.PROFILER = None
        summ = prof.summary()
        if args.layers:
            write_layers(prof, args.layers, 2)
        traffic_file = args.traffic_file
        if traffic_file is None:
            traffic_file = latest_profile("pmc_traffic_train.json")
        roof, total_ms = roofline_of(summ, args.dtype, 2, traffic_file)
        rec = {"metric": TRAIN_METRIC, "value": round(value, 2), "unit": "MPix/s",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": args.dtype,
               "data": "synthetic (seeded RGB k/255 + 4 alpha patterns; random-init weights, "
                       "torch seed 234)",
               "config": {"workload": "trainRGB.py step: AutoEncoderRGB_Journal forward + "
                                      "backward of 4096*mse+bpp + clamp(+-5) + Adam "
                                      f"(BASELINE config {3 if world == 1 else 5}), {S}x{S} RGBA",
                          "global_batch": B * world, "per_gpu_batch": B, "height": S,
                          "width": S, "parallelism": f"dp{world}", "hip_graph": captured,
                          "tile_cache": tuned and os.path.relpath(tuned, ROOT),
                          "loss": round(loss_val, 4)},
               "roofline": roof}
        if args.kernels:
            rec["kernels"] = {k: {"launches": v["launches"] // 2, "ms": round(v["ms"] / 2, 4),
                                  "share": round(v["ms"] / total_ms, 4),
                                  "tflops": round(v["flops"] / max(v["ms"], 1e-9) / 1e9, 2)}
                              for k, v in sorted(summ.items(), key=lambda kv: -kv[1]["ms"])}
        rec["cpu_baseline"] = None
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline_train(args.cpu_seconds)
        print(json.dumps(rec), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def capture_train(step, opt, dev, no_graph, before=None):
    """Capture one training step (forward, backward, all-reduces, clamp + Adam) in a HIP
    graph: Adam switches to its device step counter, two warm steps run on a side stream
    (the capture stream's allocations and autograd nodes), then the capture.  ``before``:
    called right before the captured step (e.g. to arm timing events).  Returns
    (run, graph, captured output); (step, None, None) with ``no_graph``."""
    if no_graph:
        return step, None, None
    opt.use_device_step()
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(2):
            step()
    torch.cuda.current_stream(dev).wait_stream(side)
    if before is not None:
        before()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        gout = step()
    torch.cuda.synchronize()

    def run():
        graph.replay()
        return gout
    for _ in range(2):
        run()
    torch.cuda.synchronize()
    return run, graph, gout


def dp_train_record(args, world, rank, dev, dist):
    """BASELINE config 5 inside the driver's own scaling command: the trainRGB.py step
    (forward + backward of 4096*mse + bpp, clamp(+-5), Adam) at 16 images per rank, 256^2, bf16,
    data-parallel over the ranks of THIS run -- bucketed all-reduce of the 34 M fp32 gradients
    (RCCL called directly, rgbac.parallel.RcclComm) launched from post-accumulate-grad hooks
    (rgbac.parallel.DataParallelTrainer),
    the step captured in a HIP graph (RCCL collectives included) and replayed.  At world 1
    (plain ``python bench.py``) a one-rank RCCL process group is created and the buckets are
    forced on, so the 1-rank and N-rank numbers run the same code path: same backward, same
    hook-launched all-reduces, same graph.  Every rank calls this (collectives); rank 0 gets
    the record.  ``exposed_allreduce_ms``: replayed-step time minus that of the same step
    captured without the all-reduces (what backward did not hide); ``allreduce_ms`` the same
    136 MB reduced alone."""
    import torch.distributed as tdist
    from rgbac.layers.SupplyMask import mask_pyramid
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    from rgbac.optim import AdamClamp
    from rgbac.parallel import CommWatchdog, DataParallelTrainer, RcclComm
    from rgbac import runtime as rt
    own_group = False
    if not tdist.is_initialized():
        # plain `python bench.py`: one rank, an in-process store, RCCL communicator of one
        from rgbac.parallel import _stdout_to_stderr
        with _stdout_to_stderr():       # RCCL's version banner: stderr, not the JSON line
            tdist.init_process_group("nccl", store=tdist.HashStore(), rank=0, world_size=1,
                                     device_id=dev)
        own_group = True
    B, S = args.dp_batch, 256
    tuned = os.path.join(ROOT, "profiles", f"tune_train_bf16_b{B}_{S}.json")
    if os.path.exists(tuned):
        rt.load_tune_cache(tuned)
    torch.manual_seed(234)
    net = AutoEncoder().train().to(dev).set_compute_dtype(torch.bfloat16)
    opt = AdamClamp(net.parameters(), lr=1e-4, clip=5.0)
    trainer = DataParallelTrainer(net, opt, force_buckets=True)
    x, a = synth_inputs(B, S, S, seed=1000 + rank)     # this rank's shard of the global batch
    x, a = x.to(dev), a.to(dev)
    _, me = mask_pyramid(a, 4)

    def step():
        out = net(x, a, a, *me)
        loss = 4096.0 * out[1] + out[2]                 # trainRGB.py:183-186 (lambda 4096)
        trainer.step(loss)
        return loss.detach()

    trainer_rccl = trainer.buckets.comm is not None
    # failure detection: a dead peer leaves every survivor blocked in a collective; the
    # watchdog aborts the communicator and exits non-zero once an armed stretch overruns its
    # deadline.  Armed per stretch (learning step and warmup included), the deadline scaled
    # to the stretch's steps; stopped on every exit path
    wd = CommWatchdog(trainer.buckets.comm, timeout_s=240.0).start() if trainer_rccl else None

    class _armed:
        def __init__(self, nsteps):
            self.n = nsteps

        def __enter__(self):
            if wd is not None:
                wd.timeout_s = 120.0 + 10.0 * self.n
                wd.arm()

        def __exit__(self, *exc):
            if wd is not None:
                if exc[0] is None:
                    torch.cuda.synchronize()
                wd.disarm()
            return False

    try:
        with _armed(max(1, args.dp_warmup)):
            step()                                      # learning step of the buckets
            for _ in range(max(0, args.dp_warmup - 1)):
                step()
        nb = len(trainer.buckets.buckets)
        launched = trainer.buckets.launched_in_backward()
        graph_err = None
        with _armed(4):
            try:
                run, graph, gout = capture_train(step, opt, dev, args.no_graph)
            except RuntimeError as e:                   # recorded, the eager step is timed
                graph_err = f"{type(e).__name__}: {str(e)[:200]}"
                run, graph, gout = step, None, None
            for _ in range(2):
                run()
        with _armed(args.dp_steps):
            elapsed = time_steps(run, args.dp_steps, dist, dev)
        # exposed all-reduce time = what backward did not hide: the same step captured once
        # more with the bucket all-reduces left out (GradBuckets.skip), the two graphs replayed
        # in alternation, HIP events around the replays on the replaying stream (timing events
        # cannot be recorded inside a capture on ROCm).  Measured after the timed loop: the
        # comm-free replays update each rank's replica with its own gradient only.  At world 1
        # the all-reduce moves nothing over xGMI, so no overlap is reported there.
        exposed = None
        n_ranks = tdist.get_world_size()
        if graph is not None and n_ranks > 1:
            with _armed(30):
                trainer.buckets.skip = True
                try:
                    run_nc, graph_nc, _ = capture_train(step, opt, dev, False)
                finally:
                    trainer.buckets.skip = False
                t_dp, t_nc = [], []
                for _ in range(4):
                    for fn, acc in ((run, t_dp), (run_nc, t_nc)):
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        e0.record()
                        for _ in range(3):
                            fn()
                        e1.record()
                        e1.synchronize()
                        acc.append(e0.elapsed_time(e1) / 3)
                exposed = max(0.0, min(t_dp) - min(t_nc))
                del run_nc, graph_nc
        with _armed(10):
            loss_val = run()
            finite = bool(torch.isfinite(loss_val).item())
            flat = opt.flat_grad
            for _ in range(2):
                trainer.buckets.allreduce_all()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                trainer.buckets.allreduce_all()
            e1.record()
            torch.cuda.synchronize()
            ar_ms = e0.elapsed_time(e1) / 5
            t = torch.tensor([-1.0 if exposed is None else exposed, ar_ms], device=dev,
                             dtype=torch.float64)
            tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        exposed, ar_ms = t.tolist()
        exposed = None if exposed < 0 else exposed
        rccl_ranks = trainer.buckets.comm.count() if trainer_rccl else None
    finally:
        if wd is not None:
            wd.disarm()
            wd.stop()
    grad_bytes = flat.numel() * flat.element_size()
    trainer.buckets.remove()
    del run, graph, gout, net, opt, trainer
    if own_group:
        RcclComm.close_all()
        tdist.destroy_process_group()
    if rank != 0:
        return None
    return {"metric": TRAIN_METRIC, "config": "BASELINE config 5 (config 3 at world 1): "
            f"data-parallel trainRGB.py step, {B}/rank x {n_ranks} ranks, {S}x{S}, bf16, the "
            "same code path at every world size: bucketed RCCL all-reduce launched from "
            "post-accumulate-grad hooks during backward, step captured in a HIP graph",
            "value": round(n_ranks * B * S * S * args.dp_steps / elapsed / 1e6, 3), "unit": "MPix/s",
            "n_ranks": n_ranks, "rccl_ranks": rccl_ranks, "global_batch": B * n_ranks, "steps": args.dp_steps,
            "warmup": args.dp_warmup, "ms_per_step": round(elapsed / args.dp_steps * 1e3, 3),
            "backend": "RCCL (direct ncclAllReduce on a comm stream, csrc/comm.cpp)"
            if trainer_rccl else "torch.distributed", "hip_graph": graph_err is None and not args.no_graph,
            "graph_error": graph_err, "buckets": nb, "buckets_launched_in_backward": launched,
            "exposed_allreduce_ms": None if exposed is None else round(exposed, 4),
            "allreduce_ms": round(ar_ms, 4), "gradient_bytes": grad_bytes,
            "overlap_fraction": None if (exposed is None or ar_ms <= 0)
            else round(min(1.0, max(0.0, 1 - exposed / ar_ms)), 3),
            "loss_finite": finite}


def cpu_baseline_codec(budget_s):
    """Oracle compress (CPU fp32 symbols + the pure-Python rANS restatement) on 1 image."""
    from oracle import ans_ref as oa
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    cores = _set_cpu_threads()
    torch.manual_seed(234)
    net = AutoEncoder().eval()
    net.update()
    sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    gc = net.gaussian_conditional
    tab = (gc.quantized_cdf.tolist(), gc.cdf_length.tolist(), gc.offset.tolist())
    x, a = synth_inputs(2, 256, 256, seed=0)
    x, a = x[1:2], a[1:2]
    n, t0 = 0, time.perf_counter()
    while True:
        with torch.no_grad():
            _, syms, idxs, _ = oa.rgb_compress_symbols(sd, x, a, gc.scale_table)
        enc = oa.BufferedRansEncoder()
        enc.encode_with_indexes(torch.cat([s.reshape(-1) for s in syms]).tolist(),
                                torch.cat([i.reshape(-1) for i in idxs]).tolist(), *tab)
        enc.flush()
        n += 1
        if time.perf_counter() - t0 >= budget_s or n >= 100:
            break
    dt = time.perf_counter() - t0
    return {"value": round(n * 256 * 256 / dt / 1e6, 4), "unit": "MPix/s",
            "cores": cores, "kind": "port",
            "sample": f"oracle compress (fp32 symbols + pure-Python rANS of y), 1 image "
                      f"256x256 (half-transparent alpha), {n} iterations, {dt:.1f} s"}


def main_codec(args, dev):
    """--codec: AutoEncoder.compress + decompress (AutoEncoderRGB_Journal.py:312-416) end to
    end: GPU transforms + symbol/index kernels, device<->host copies, host rANS coder."""
    from rgbac.layers.SupplyMask import mask_pyramid
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    torch.manual_seed(234)
    net = AutoEncoder().eval().to(dev).set_compute_dtype(dt)
    net.update()
    B, S = args.batch, args.size
    x, a = synth_inputs(B, S, S, seed=0)
    x, a = x.to(dev), a.to(dev)
    for _ in range(max(args.warmup, 1)):
        out = net.compress(x, a)
        rec = net.decompress(out["strings"], out["shape"], a)
    torch.cuda.synchronize()
    tc, td = [], []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        out = net.compress(x, a)
        t1 = time.perf_counter()
        rec = net.decompress(out["strings"], out["shape"], a)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        tc.append(t1 - t0)
        td.append(t2 - t1)
    tc.sort()
    td.sort()
    mc, md = tc[len(tc) // 2], td[len(td) // 2]
    nbytes = sum(len(s) for s in out["strings"][0]) + sum(len(s) for s in out["strings"][1])
    _, me = mask_pyramid(a, 4)
    with torch.no_grad():
        fwd = net(x, a, a, *me)
    npx = B * S * S
    rec = {"metric": "MPixels/sec compress+decompress (real rANS bitstream), 256x256 RGBA batch",
           "value": round(npx / (mc + md) / 1e6, 3), "unit": "MPix/s", "n_gpus": 1,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round((mc + md) * 1e3, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
           "data": "synthetic (seeded RGB k/255 + 4 alpha patterns; random-init weights)",
           "config": {"workload": f"AutoEncoderRGB_Journal compress + decompress, {S}x{S}",
                      "batch": B},
           "compress_ms": round(mc * 1e3, 3), "decompress_ms": round(md * 1e3, 3),
           "compress_mpix_s": round(npx / mc / 1e6, 3), "decompress_mpix_s": round(npx / md / 1e6, 3),
           "actual_bpp": round(8 * nbytes / npx, 5), "estimated_bpp": round(fwd[2].item(), 5),
           "cpu_baseline": None}
    if not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline_codec(args.cpu_seconds)
    print(json.dumps(rec), flush=True)


def cpu_baseline_rgba(budget_s):
    """Oracle alpha codec + constraint + RGB codec (trainRGB.py:282-306) on 1 image, fp32."""
    from oracle import ref_model as ref
    from rgbac.models.AutoEncoderMask_Journal import AutoEncoder as MaskNet
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder as RGBNet
    cores = _set_cpu_threads()
    torch.manual_seed(234)
    sdr = {k: v.detach() for k, v in RGBNet().state_dict().items()}
    sdm = {k: v.detach() for k, v in MaskNet().state_dict().items()}
    x, a = synth_inputs(2, 256, 256, seed=0)
    x, a = x[1:2], a[1:2]
    n, t0 = 0, time.perf_counter()
    while True:
        with torch.no_grad():
            ref.rgba_forward(sdm, sdr, x, a)
        n += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": round(n * 256 * 256 / dt / 1e6, 4), "unit": "MPix/s",
            "cores": cores, "kind": "port",
            "sample": f"oracle rgba_forward fp32 (alpha codec + constraint + RGB codec), 1 image "
                      f"256x256 (half-transparent alpha), {n} iterations, {dt:.1f} s"}


def main_rgba(args, dev):
    """--rgba: the RGBA evaluation pipeline (trainRGB.py:282-306): alpha
    codec forward -> clamp/round/constraint -> RGB codec forward -> clamp + bpp/PSNR, all on
    the GPU, one HIP graph per step."""
    from rgbac.models.AutoEncoderMask_Journal import AutoEncoder as MaskNet
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder as RGBNet
    from rgbac.rgba import rgba_forward
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    torch.manual_seed(234)
    net = RGBNet().eval().to(dev).set_compute_dtype(dt)
    msk = MaskNet().eval().to(dev).set_compute_dtype(dt)
    B, S = args.batch, args.size
    x, a = synth_inputs(B, S, S, seed=0)
    x, a = x.to(dev), a.to(dev)

    def step():
        return rgba_forward(msk, net, x, a)

    step()
    torch.cuda.synchronize()
    run = step
    if not args.no_graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                step()
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = step()
        run = graph.replay
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if args.no_graph:
        out = step()
    # eval metric of the same loop (trainRGB.py:311), outside the timed codec region as there
    from rgbac.metrics.ms_ssim_torch import ms_ssim
    msv = ms_ssim(x, out[0], data_range=1.0).item()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        ms_ssim(x, out[0], data_range=1.0)
    torch.cuda.synchronize()
    ms_ms = (time.perf_counter() - t0) / 10 * 1e3
    npx = B * S * S
    rec = {"metric": "MPixels/sec RGBA encode+decode (alpha codec -> constraint -> RGB codec)",
           "value": round(npx * args.steps / el / 1e6, 3), "unit": "MPix/s", "n_gpus": 1,
           "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
           "data": "synthetic (seeded RGB k/255 + 4 alpha patterns; random-init weights)",
           "config": {"workload": f"RGBA eval pipeline trainRGB.py:282-306, {S}x{S}",
                      "batch": B, "hip_graph": not args.no_graph},
           "bpp": round(out[3].item(), 5), "psnr": round(out[4].item(), 4),
           "ms_ssim": round(msv, 6), "ms_ssim_ms_per_batch": round(ms_ms, 3),
           "cpu_baseline": None}
    if not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline_rgba(args.cpu_seconds)
    print(json.dumps(rec), flush=True)


def main_alpha(args, dev):
    """--alpha: BASELINE config 1 -- AutoEncoderMask_Journal encode+decode of one 256x256 alpha
    tile (trainmask.py:242-293, config4096.json), HIP graph replay, in the bench dtype and in
    fp32; cpu_baseline = the oracle's mask_forward on the same tile (the reference runs this
    config on PyTorch CPU); parity (fp32, teacher-forced symbol accounting) vs the oracle."""
    from oracle import parity as opar
    from oracle import ref_model as ref
    from rgbac import runtime as rt
    from rgbac.models._latent import debug_views
    B, S = args.batch if "--batch" in sys.argv else 1, args.size
    _, a = synth_inputs(max(B, 4), S, S, seed=0)
    a = a[2:3].repeat(B, 1, 1, 1) if B == 1 else a[:B]     # the ramped-ellipse alpha tile
    net = mask_net().to(dev)
    sd = {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}
    ad = a.to(dev)
    res = {}
    for dtn in ([args.dtype, "f32"] if args.dtype != "f32" else ["f32"]):
        net.set_compute_dtype(torch.bfloat16 if dtn == "bf16" else torch.float32)

        def step():
            with torch.no_grad():
                return net(ad)
        step()
        torch.cuda.synchronize()
        run, graph, _ = capture(step, args.no_graph)
        for _ in range(args.warmup):
            run()
        el = time_steps(run, args.steps, None, dev)
        res[dtn] = {"value": round(B * S * S * args.steps / el / 1e6, 3),
                    "ms_per_step": round(el / args.steps * 1e3, 4)}
        del run, graph
    # parity (fp32, one tile) and the CPU baseline
    net.set_compute_dtype(torch.float32)
    dbg = {}
    with torch.no_grad(), rt.fixed_tiles():
        o = net(ad[:1], debug=dbg)
    dev_out = (o[0].cpu(),) + tuple(t.item() for t in o[1:])
    rep = opar.north_star_report(sd, "mask", a[:1], None, debug_views(dbg), dev_out)
    cores = _set_cpu_threads()
    with torch.no_grad():
        r = ref.mask_forward(sd, a[:1])
        n, t0 = 0, time.perf_counter()
        while True:
            ref.mask_forward(sd, a[:1])
            n += 1
            if time.perf_counter() - t0 >= args.cpu_seconds or n >= 2000:
                break
        dt_cpu = time.perf_counter() - t0
    main = res[args.dtype]
    rec = {"metric": "MPixels/sec alpha-codec encode+decode (AutoEncoderMask_Journal), 256x256 tile",
           "value": main["value"], "unit": "MPix/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": main["ms_per_step"], "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
           "data": "synthetic (ramped-ellipse alpha k/255; random-init weights, torch seed 234, "
                   "EncoderMask.7 x20 so latent symbols are non-zero)",
           "config": {"workload": f"BASELINE config 1: AutoEncoderMask_Journal forward, {S}x{S}",
                      "batch": B, "hip_graph": not args.no_graph},
           "parity_mode": {"dtype": "f32", **res["f32"]},
           "parity": {"sample": f"the same tile, fp32, vs the CPU oracle",
                      "rel_d_bpp": float(f"{abs(dev_out[2] - r[2].item()) / r[2].item():.3g}"),
                      "d_psnr_db": float(f"{abs(opar.psnr_db(dev_out[1]) - opar.psnr_db(r[1].item())):.3g}"),
                      "max_abs_d_x_hat": float(f"{(dev_out[0] - r[0]).abs().max().item():.3g}"),
                      "symbols": rep["symbols"], "nonzero_symbols": rep["nonzero_symbols"],
                      "flips": rep["flips"], "far_flips": rep["far_flips"],
                      "tf_d_psnr_db": rep["tf_d_psnr_db"], "tf_d_ms_ssim": rep["tf_d_ms_ssim"]},
           "cpu_baseline": {"value": round(n * S * S / dt_cpu / 1e6, 4), "unit": "MPix/s",
                            "cores": cores, "kind": "port",
                            "sample": f"oracle mask_forward fp32, the same {S}x{S} tile, {n} "
                                      f"forwards, {dt_cpu:.1f} s, torch threads {cores}"}}
    print(json.dumps(rec), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--dtype", choices=["bf16", "f32"], default="bf16")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity-mode", action="store_true",
                    help="skip the fp32 parity-mode timing of the same config")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--kernels", action="store_true", help="add the per-kernel time table")
    ap.add_argument("--layers", default=None, help="write a per-layer time table to this file")
    ap.add_argument("--train", action="store_true",
                    help="time the training step (BASELINE config 3 / 5) instead of the forward")
    ap.add_argument("--rgba", action="store_true",
                    help="RGBA eval pipeline: alpha codec -> constraint -> RGB codec")
    ap.add_argument("--alpha", action="store_true",
                    help="BASELINE config 1: the alpha codec on one 256x256 tile")
    ap.add_argument("--codec", action="store_true",
                    help="time compress + decompress (real bitstream) instead of the forward")
    ap.add_argument("--tune-cache", default=None,
                    help="tile-choice cache to load (default: the committed profiles/ one for "
                         "the forward config); '' disables")
    ap.add_argument("--save-tune", default=None, help="write the tile-choice cache here")
    ap.add_argument("--no-dp-train", action="store_true",
                    help="skip the data-parallel training sub-record (config 5 / dp_train)")
    ap.add_argument("--dp-batch", type=int, default=16, help="dp_train images per rank")
    ap.add_argument("--dp-steps", type=int, default=5)
    ap.add_argument("--dp-warmup", type=int, default=3)
    ap.add_argument("--traffic-file", default=None,
                    help="PMC traffic summary (default: the committed profiles/ one)")
    args = ap.parse_args()
    if args.train and args.batch == 8 and "--batch" not in sys.argv:
        args.batch = 16

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` without a launcher: start N rank processes of this script
        # ourselves (one per GPU, the torchrun environment contract), before this process
        # touches the GPU; this parent only waits and returns the worst exit code.
        return spawn_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world and "--gpus" in sys.argv:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        from rgbac.parallel import _stdout_to_stderr
        with _stdout_to_stderr():       # RCCL's version banner: stderr, not the JSON line
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    if args.train:
        return main_train(args, world, rank, dev, dist)
    if args.codec:
        return main_codec(args, dev)
    if args.rgba:
        return main_rgba(args, dev)
    if args.alpha:
        return main_alpha(args, dev)
    return main_forward(args, world, rank, dev, dist)


def spawn_ranks(n):
    """Launch ``n`` copies of this command line as ranks 0..n-1 (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT), wait for all, return the max exit code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    if rc:
        raise SystemExit(rc)
    return 0


def capture(step, no_graph):
    """Warm ``step`` on a side stream and capture it in a HIP graph -> (run, graph, out)."""
    if no_graph:
        return step, None, None
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = step()
    return graph.replay, graph, out


def time_steps(run, steps, dist, dev):
    """Barrier + synchronize, ``steps`` timed steps, synchronize + barrier; the MAX over ranks."""
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    return elapsed


def main_forward(args, world, rank, dev, dist):
    """BASELINE config 2 (B=8, 256^2, bf16) / config 4 (--size 1024 --batch 4): forward
    encode+decode, replicas on N GPUs."""
    from rgbac import runtime as rt
    from rgbac.layers.SupplyMask import mask_pyramid
    from rgbac.models.AutoEncoderRGB_Journal import AutoEncoder

    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    net = rgb_net().to(dev).set_compute_dtype(dt)
    B, S = args.batch, args.size
    x, a = synth_inputs(B, S, S, seed=rank)
    x, a = x.to(dev), a.to(dev)
    _, me = mask_pyramid(a, 4)

    def step():
        with torch.no_grad():                          # inference: the fused, grouped path
            return net(x, a, a, *me)

    tuned = tune_cache_setup(args, os.path.join(ROOT, "profiles", f"tune_fwd_{args.dtype}_b{B}_{S}.json"))
    step()                                             # packs weights, warms caches (and tunes)
    torch.cuda.synchronize()
    run, graph, _ = capture(step, args.no_graph)
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    elapsed = time_steps(run, args.steps, dist, dev)
    ms = elapsed / args.steps * 1e3
    value = world * B * S * S * args.steps / elapsed / 1e6

    # fp32 parity mode (the reference's own precision) on the same config, timed the same way
    parity_mode = None
    if dt != torch.float32 and not args.no_parity_mode:
        if tune_cache_setup(args, os.path.join(ROOT, "profiles", f"tune_fwd_f32_b{B}_{S}.json")):
            pass
        net.set_compute_dtype(torch.float32)
        step()
        torch.cuda.synchronize()
        run32, graph32, _ = capture(step, args.no_graph)
        for _ in range(2):
            run32()
        psteps = max(3, args.steps // 4)
        el32 = time_steps(run32, psteps, dist, dev)
        del graph32, run32
        parity_mode = {"dtype": "f32", "value": round(world * B * S * S * psteps / el32 / 1e6, 2),
                       "unit": "MPix/s", "steps": psteps,
                       "ms_per_step": round(el32 / psteps * 1e3, 3),
                       "note": "same config at the reference's precision: fp32 storage, "
                               "exact-fp32 MFMA (v_mfma_f32_16x16x4_f32), fp32 epilogues"}
        net.set_compute_dtype(dt)
    if args.save_tune and rank == 0:
        rt.save_tune_cache(args.save_tune)
    # config 5 (DP training) in the same ranks, so the driver's scaling run measures it too
    dp = None
    if not args.no_dp_train:
        dp = dp_train_record(args, world, rank, dev, dist)

    if rank == 0:
        # ---- roofline attribution: eager steps, each queued behind a GPU spin so the host has
        # enqueued every launch before the GPU reaches them (back-to-back execution as in the
        # graph replay), with a fence-free HIP event (rgbac_timer_*: no cache writeback /
        # invalidate per record) on the launching stream around every launch.
        prof = rt.LaunchProfiler()
        nrep = 3
        rt.PROFILER = prof
        for _ in range(nrep):
            torch.cuda._sleep(SPIN_FWD)
            step()
            torch.cuda.synchronize()
        rt.PROFILER = None
        summ = prof.summary()
        if args.layers:
            write_layers(prof, args.layers, nrep)
        traffic_file = args.traffic_file
        if traffic_file is None:                       # a summary taken on this workload
            traffic_file = (latest_profile(f"pmc_traffic_fwd_b{B}_{S}.json") or
                            latest_profile("pmc_traffic_fwd.json"))
        roof, total_ms = roofline_of(summ, args.dtype, nrep, traffic_file,
                                     {"batch": B, "size": S, "dtype": args.dtype})
        roof["timing"] = "eager steps behind a GPU spin, fence-free HIP events per launch"
        if roof["traffic"] is not None:
            roof["traffic_source"] = os.path.relpath(traffic_file, ROOT)
        fwd_flops = sum(d["flops"] for d in summ.values()) / nrep
        rec = {"metric": METRIC, "value": round(value, 2), "unit": "MPix/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": args.dtype, "data": "synthetic (seeded RGB k/255 + 4 alpha patterns; "
                                             "random-init weights, torch seed 234, Encoder.x4 "
                                             "x20 so latent symbols are non-zero)",
               "config": {"workload": "AutoEncoderRGB_Journal forward encode+decode "
                                      f"(BASELINE config {2 if S == 256 else 4}), {S}x{S} RGBA",
                          "global_batch": B * world, "per_gpu_batch": B, "height": S, "width": S,
                          "parallelism": f"replicas{world}", "hip_graph": graph is not None,
                          "tile_cache": tuned and os.path.relpath(tuned, ROOT)},
               "roofline": roof,
               "achieved_model_tflops": round(fwd_flops / (ms * 1e-3) / 1e12, 2),
               "parity_mode": parity_mode, "dp_train": dp}
        if args.kernels:
            rec["kernels"] = {k: {"launches": v["launches"] // nrep, "ms": round(v["ms"] / nrep, 4),
                                  "share": round(v["ms"] / total_ms, 4),
                                  "tflops": round(v["flops"] / max(v["ms"], 1e-9) / 1e9, 2)}
                              for k, v in sorted(summ.items(), key=lambda kv: -kv[1]["ms"])}
        rec["cpu_baseline"] = None
        rec["parity"] = None
        if world == 1 and not args.no_cpu_baseline:
            # the CPU baseline and parity sample are the bench's own size (config 4: 1024^2)
            rec["cpu_baseline"], outs_ref = cpu_baseline(args.cpu_seconds, S=S)
            # bpp / PSNR / MS-SSIM of the HIP forward vs the oracle on the same sample
            # (outside the timed region), in the bench dtype and in the fp32 parity mode
            par = {"sample": f"4 images {S}x{S} of the bench batch (alpha ones / half / "
                             "ellipse / zero), one forward each, vs the CPU oracle (fp32)"}
            par[args.dtype] = gpu_parity(net, dev, outs_ref, S=S, account=dt == torch.float32)
            if dt != torch.float32:
                net.set_compute_dtype(torch.float32)
                par["f32"] = gpu_parity(net, dev, outs_ref, S=S, account=True)
                net.set_compute_dtype(dt)
            rec["parity"] = par
        print(json.dumps(rec), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
