"""Throughput bench of the north-star path: res15 eval forward over synthetic
[B,101,40] fp32 MFCC maps resident in HBM, on the gfx950 kernels.

    python bench.py [--gpus N --steps K --warmup W --batch B]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

One step = one forward of B clips per GPU (weak scaling: per-GPU batch fixed;
the batch shards across ranks with no collective on the data path).  Prints ONE
JSON line on rank 0 (see DESIGN.md "Measurement").
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "1s-clips/sec (whole node) + top-1 acc, res15 12-label Speech Commands"
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_*_f32 dense peak (= FP32 vector peak)
HBM_PEAK_GBS = 8000.0
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (no sparsity)
WORKLOADS = {
    "res15": "res15 eval forward (SpeechResModel, 13 dilated 3x3 res layers, 45 maps, 12 labels)",
    "res8": "res8 eval forward (SpeechResModel, avg-pool 4x3, 6 res layers, 45 maps, 12 labels)",
    "cnn-trad-pool2": "cnn-trad-pool2 eval forward (SpeechModel, conv 20x8 + maxpool 2x2 + conv 10x4 + linear, 4 labels)",
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--batch", type=int, default=None,
                   help="clips per GPU per step (default: res* 131072 = C4's 1M over 8 GPUs; cnn* 65536 = C2)")
    p.add_argument("--model", default="res15")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--precision", default="bf16x3", choices=["bf16x3", "f32", "bf16"],
                   help="res path arithmetic: bf16x3 (fp32 values as bf16 hi/lo pairs, 3 bf16 MFMA products, "
                        "fp32 accumulation; 1e-4 parity), f32 (fp32 MFMA; 1e-4 parity) or bf16 (top-1 parity)")
    p.add_argument("--no-alt", action="store_true",
                   help="skip the extra measurements of the other res precision modes")
    p.add_argument("--e2e", action="store_true",
                   help="serving pipeline: int16-scaled PCM [B,16000] in HBM -> GPU MFCC -> model -> logits")
    p.add_argument("--train", action="store_true",
                   help="C5: data-parallel training step (fwd+bwd, one RCCL all-reduce, fused SGD)")
    return p.parse_args()


def cpu_baseline(cfg, seconds):
    """The reference's CPU path restated (oracle/ref_torch.py: stock torch fp32 eval
    forward, what utils/train.py --no_cuda runs) on the host cores: bounded sample.
    Threads = the box's CPU share (16 on the GPU pool; os.cpu_count() shows the
    whole machine there), batches as SURVEY.md §8(d): 64 clips for res15, else 256."""
    import torch
    from oracle import ref_numpy as orc
    from oracle import ref_torch
    cores = int(os.environ.get("OMP_NUM_THREADS") or 0) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(cores)
    params = ref_torch.tensors(orc.make_params(cfg, 0))
    rng = np.random.Generator(np.random.PCG64(1))
    per = 64 if int(cfg.get("n_layers", 0)) > 8 else 256
    x = torch.from_numpy(rng.standard_normal((per, 101, 40)).astype(np.float32))
    ref_torch.forward(params, cfg, x[:2])  # warm-up
    ref_torch.forward(params, cfg, x)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        ref_torch.forward(params, cfg, x)
        n += per
    dt = time.perf_counter() - t0
    model_name = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            model_name = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), model_name)
    except OSError:  # pragma: no cover
        pass
    return {"value": n / dt, "unit": "clips/s", "cores": int(cores), "kind": "port",
            "sample": f"{n} clips of {cfg_name(cfg)} in {dt:.1f} s (oracle/ref_torch.py: torch {torch.__version__} "
                      f"CPU fp32 eval forward, batches of {per}, {cores} threads)",
            "cpu_model": model_name, "os_cpu_count": os.cpu_count()}


def cfg_name(cfg):
    if "n_layers" not in cfg:
        return "cnn"
    return (f"res (n_layers {cfg['n_layers']}, {cfg['n_feature_maps']} maps"
            f"{', dilated' if cfg.get('use_dilation') else ''})")


def load_traffic(kernel, clips_per_launch, model):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 PMC pass
    (profiles/pmc_<kernel>.json, written by tools/pmc_summary.py), or None when no
    pass was taken for that kernel at this launch size."""
    p = os.path.join(REPO, "profiles", f"pmc_{kernel}.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
    except Exception:
        return None
    if d.get("batch_clips_per_launch") != clips_per_launch or d.get("model") != model:
        return None
    return d.get("hbm_bytes_per_launch")


def train_bench(args, dev, rank, world, barrier):
    """C5: res26-narrow train step per rank (fwd+bwd on device, flat-bucket all-reduce, fused SGD)."""
    from honk_amd import distributed as hd
    from honk_amd import model as hm
    from honk_amd.optim import FlatParams, FlatSGD
    name = args.model if args.model != "res15" else "res26-narrow"
    B = args.batch or 4096
    cfg = dict(hm.find_config(name))
    torch.manual_seed(0)
    model = hm.find_model(name)(cfg).to(dev).train()
    hd.broadcast_module(model)
    flat = FlatParams(model)
    opt = FlatSGD(flat, lr=0.1, momentum=0.9, weight_decay=1e-5)
    crit = torch.nn.CrossEntropyLoss()
    g = torch.Generator(device=dev).manual_seed(99 + rank)
    x = torch.randn(B, 101, 40, device=dev, generator=g)
    y = torch.randint(0, cfg["n_labels"], (B,), device=dev, generator=g)

    def step():
        opt.zero_grad()
        hd.broadcast_module(model, buffers_only=True)
        loss = crit(model(x), y)
        loss.backward()
        opt.step(grad_scale=hd.allreduce_grads(flat))
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = hd.max_over_ranks(t1 - t0, device=dev)
    value = world * B * args.steps / elapsed
    if rank == 0:
        print(json.dumps({
            "metric": "train clips/sec (whole node), res26-narrow fwd+bwd+SGD, DP over RCCL (config C5)",
            "value": round(value, 1), "unit": "clips/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic N(0,1) [B,101,40] inputs + uniform labels resident in HBM",
            "config": {"workload": f"{name} training step (train mode BN batch stats, CE loss, SGD m=0.9)",
                       "per_gpu_batch": B, "global_batch": world * B,
                       "parallelism": f"dp{world}: one flat fp32 grad bucket all-reduce ({flat.numel} params)"},
            "final_loss": float(loss.item()),
            "roofline": None,
            "note": "native kernels: the block convs' forward / input grad / weight grad "
                    "(honk_conv3x3_f32, honk_conv3x3_wgrad_f32), train-mode BatchNorm fwd/bwd "
                    "(honk_bn_train_*), fused SGD over the flat all-reduced bucket; conv0, pooling, ReLU, "
                    "residual, mean, Linear and the loss run on PyTorch autograd on the device"}),
              flush=True)


def _res_geometry(cfg):
    """(H, W, n_layers, CP) of a res config's block layers (model.py:87-98)."""
    ph, pw = tuple(cfg.get("res_pool", (1, 1)))
    C = int(cfg["n_feature_maps"])
    return 101 // ph, 40 // pw, int(cfg["n_layers"]), 16 * ((C + 15) // 16)


PREC_NOTES = {
    "bf16x3": "fp32 values carried as bf16 (hi, lo) pairs; products hi*hi + hi*lo + lo*hi on bf16 MFMA, fp32 "
              "accumulation; meets the fp32 1e-4 logit parity bar (tests/test_gpu_bf16x3.py)",
    "f32": "IEEE fp32 on v_mfma_f32_16x16x4_f32; 1e-4 logit parity",
    "bf16": "bf16 activations/weights, fp32 accumulation; top-1 parity only (reduced precision vs the fp32 "
            "reference), so never the headline",
}


def res_roofline(prec, cfg, kms, nl, kfl, B, model):
    """Roofline of the dominant res kernel for a precision mode.

    f32: MFMA-bound -- algorithmic FLOP per launch / mean launch time vs the fp32
    MFMA peak.  bf16 / bf16x3 (block16_kernel, SP = 1 / 2): HBM-bound --
    algorithmic bytes per launch = clips x (read X [+ read residual on even layers]
    [+ write Y except the last layer]) x H*W*CP*2*SP, averaged over the layers of
    one forward, / the mean launch time."""
    avg_s = (kms / max(nl, 1)) * 1e-3
    clips = min(B, 4096)
    if prec == "f32":
        ach = (kfl / max(nl, 1)) / avg_s / 1e12 if nl else None
        return {"bound": "mfma", "kernel": "honk::res::block_kernel (dilated 3x3 conv, fp32 MFMA)",
                "achieved": round(ach, 2) if ach else None, "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4) if ach else None,
                "traffic": load_traffic("block_kernel", clips, model),
                "launches": nl, "avg_launch_ms": round(kms / max(nl, 1), 4),
                "flop_per_launch": kfl / max(nl, 1)}
    sp = 2 if prec == "bf16x3" else 1
    H, W, L, CP = _res_geometry(cfg)
    act = H * W * CP * 2 * sp
    per_clip = sum(act * (1 + (1 if i % 2 == 0 else 0) + (1 if i < L else 0)) for i in range(1, L + 1)) / L
    bw = per_clip * clips / avg_s / 1e9 if nl else None
    mf = (kfl * (3 if sp == 2 else 1) / max(nl, 1)) / avg_s / 1e12 if nl else None
    # every res config runs the row-band kernel (HONK_RES_ROWBAND=0: the per-dy-stage one)
    fam = "block16_kernel" if os.environ.get("HONK_RES_ROWBAND") == "0" else "block16r_kernel"
    return {"bound": "hbm", "kernel": f"honk::res::{fam}<..., SP={sp}> (dilated 3x3 conv, bf16 MFMA)",
            "achieved": round(bw, 1) if bw else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(bw / HBM_PEAK_GBS, 4) if bw else None,
            "traffic": load_traffic(f"{fam}_sp{sp}", clips, model),
            "launches": nl, "avg_launch_ms": round(kms / max(nl, 1), 4),
            "algorithmic_bytes_per_launch": per_clip * clips,
            "mfma": {"executed_bf16_tflops": round(mf, 2) if mf else None, "peak": BF16_MFMA_PEAK_TFLOPS,
                     "frac": round(mf / BF16_MFMA_PEAK_TFLOPS, 4) if mf else None}}


def measure_mode(prec, model, x, args, dev, barrier, hd, _native, orc, cfg, B, world):
    """The same res workload in another precision mode (reported beside the headline)."""
    keep = model.honk_precision
    model.honk_precision = prec
    with torch.no_grad():
        for _ in range(max(1, args.warmup)):
            model(x)
        torch.cuda.synchronize()
        barrier()
        _native.timing_enable(True)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = model(x)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        barrier()
        kms, nl, kfl = _native.timing_read()
        _native.timing_enable(False)
    model.honk_precision = keep
    el = hd.max_over_ranks(t1 - t0, device=dev)
    idx = list(range(0, B, max(1, B // 32)))[:32]
    ref = orc.forward({k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}, cfg,
                      x[idx].cpu().numpy())
    got = out[idx].cpu().numpy()
    return {"value": round(world * B * args.steps / el, 1), "unit": "clips/s", "dtype": prec,
            "ms_per_step": round(el / args.steps * 1e3, 3),
            "roofline": res_roofline(prec, cfg, kms, nl, kfl, B, args.model),
            "parity": {"top1_agreement_vs_oracle": float(np.mean(ref.argmax(1) == got.argmax(1))),
                       "max_abs_logit_err_vs_oracle_f64": float(np.abs(ref - got).max()),
                       "sample_clips": len(idx)},
            "note": PREC_NOTES[prec]}


def measure_c2(args, dev, barrier, hd, _native, orc, world, rank):
    """Config C2 (BASELINE.json configs[1]): cnn-trad-pool2 eval forward, 65,536
    clips per GPU, in bf16x3 (1e-4 parity) and fp32 MFMA, reported beside the res15
    headline.  Roofline: algorithmic conv FLOP per launch over the conv kernels'
    mean launch time (HIP events on the launch stream), vs bf16 peak / 3 (bf16x3)
    or the fp32 MFMA peak."""
    from honk_amd import model as hm
    name = "cnn-trad-pool2"
    cfg = dict(hm.find_config(name))
    torch.manual_seed(0)
    model = hm.find_model(name)(cfg).eval().to(dev)
    B = 65536
    g = torch.Generator(device=dev).manual_seed(4321 + rank)
    x = torch.randn(B, 101, 40, device=dev, generator=g)
    out = {"workload": "cnn-trad-pool2 eval forward (config C2), 65,536 clips per GPU", "per_gpu_batch": B}
    for prec in ("bf16x3", "f32"):
        model.honk_precision = prec
        with torch.no_grad():
            for _ in range(max(1, args.warmup)):
                model(x)
            torch.cuda.synchronize()
            barrier()
            _native.timing_enable(True)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                y = model(x)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            barrier()
            kms, nl, kfl = _native.timing_read()
            _native.timing_enable(False)
        el = hd.max_over_ranks(t1 - t0, device=dev)
        idx = list(range(0, B, B // 32))[:32]
        ref = orc.forward({k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}, cfg,
                          x[idx].cpu().numpy())
        got = y[idx].cpu().numpy()
        peak = FP32_MFMA_PEAK_TFLOPS if prec == "f32" else BF16_MFMA_PEAK_TFLOPS / 3
        ach = (kfl / max(nl, 1)) / (kms / max(nl, 1) * 1e-3) / 1e12 if nl else None
        out[f"{prec}_mode"] = {
            "value": round(world * B * args.steps / el, 1), "unit": "clips/s", "dtype": prec,
            "ms_per_step": round(el / args.steps * 1e3, 3),
            "roofline": {"bound": "mfma",
                         "kernel": ("honk::cnn::conv1x3_kernel + conv2x3_kernel (bf16x3 convs, 3 bf16 MFMA "
                                    "products per MAC; peak = bf16 peak / 3)" if prec == "bf16x3" else
                                    "honk::cnn::conv_gemm_kernel<.., X3=false> (implicit-GEMM convs, fp32 MFMA)"),
                         "achieved": round(ach, 2) if ach else None, "peak": round(peak, 1), "unit": "TFLOP/s",
                         "frac": round(ach / peak, 4) if ach else None, "launches": nl,
                         "avg_launch_ms": round(kms / max(nl, 1), 4), "flop_per_launch": kfl / max(nl, 1)},
            "parity": {"top1_agreement_vs_oracle": float(np.mean(ref.argmax(1) == got.argmax(1))),
                       "max_abs_logit_err_vs_oracle_f64": float(np.abs(ref - got).max()),
                       "sample_clips": len(idx)},
            "note": PREC_NOTES.get(prec, "")}
    del x
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        # rehearsal knobs for a 1-GPU box (never set by the driver): HONK_BENCH_BACKEND=gloo
        # and HONK_BENCH_ONE_GPU=1 run N ranks on cuda:0 over gloo; the real N-GPU run is RCCL
        if os.environ.get("HONK_BENCH_ONE_GPU"):
            local = 0
        backend = os.environ.get("HONK_BENCH_BACKEND", "nccl")
        torch.cuda.set_device(local)
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from honk_amd import _native
    from honk_amd import distributed as hd
    from honk_amd import model as hm
    from oracle import ref_numpy as orc

    def barrier():
        if dist:
            tdist.barrier()

    if args.train:
        train_bench(args, dev, rank, world, barrier)
        if dist:
            tdist.destroy_process_group()
        return

    cfg = dict(hm.find_config(args.model))
    torch.manual_seed(0)
    model = hm.find_model(args.model)(cfg).eval().to(dev)
    is_res = args.model.startswith("res")
    if not is_res and args.precision == "bf16":
        raise SystemExit("cnn models: --precision f32 or bf16x3")
    model.honk_precision = args.precision
    B = args.batch or (131072 if is_res else 65536)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    x = torch.randn(B, 101, 40, device=dev, generator=g)  # resident in HBM before timing
    step_fn = model
    if args.e2e:  # raw 1 s PCM windows instead of MFCC maps; MFCC runs on the GPU inside the step
        from honk_amd.audio import AudioPreprocessor
        ap = AudioPreprocessor()
        pcm = (torch.rand(B, 16000, device=dev, generator=g) * 2 - 1) * 0.3
        x = pcm

        def step_fn(p):
            return model(ap.compute_mfccs_batch(p))

    with torch.no_grad():
        for _ in range(args.warmup):
            step_fn(x)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        _native.timing_enable(True)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = step_fn(x)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        barrier()
        kms, nlaunch, kflop = _native.timing_read()
        _native.timing_enable(False)
    elapsed = hd.max_over_ranks(t1 - t0, device=dev)  # whole-job time = slowest rank

    prec = args.precision
    # cnn bf16x3: each algorithmic MAC is 3 bf16 MFMA products -> effective peak = bf16 peak / 3
    peak = FP32_MFMA_PEAK_TFLOPS if prec == "f32" else BF16_MFMA_PEAK_TFLOPS / 3
    # top-1 agreement / max logit error of the GPU logits vs the float64 oracle on a sample
    idx = list(range(0, B, max(1, B // 32)))[:32]
    xs = (ap.compute_mfccs_batch(x[idx]) if args.e2e else x[idx]).cpu().numpy()
    ref = orc.forward({k: v.detach().cpu().numpy() for k, v in model.state_dict().items()},
                      cfg, xs)
    got = out[idx].cpu().numpy()
    top1 = float(np.mean(np.argmax(ref, 1) == np.argmax(got, 1)))
    maxerr = float(np.abs(ref - got).max())

    # the other precision modes of the same workload, reported beside the headline
    alts = {}
    if is_res and not args.no_alt and not args.e2e:
        for other in ("f32", "bf16"):
            if other != prec:
                alts[f"{other}_mode"] = measure_mode(other, model, x, args, dev, barrier, hd, _native, orc, cfg,
                                                     B, world)

    c2 = None
    if is_res and not args.no_alt and not args.e2e:
        c2 = measure_c2(args, dev, barrier, hd, _native, orc, world, rank)

    total = world * B * args.steps
    value = total / elapsed
    flop_clip = orc.flops_per_clip(cfg)
    avg_ms = kms / max(nlaunch, 1)
    achieved = (kflop / max(nlaunch, 1)) / (avg_ms * 1e-3) / 1e12 if nlaunch else None
    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "clips/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": prec,
            "precision_note": PREC_NOTES[prec],
            "data": "synthetic N(0,1) [B,101,40] fp32 MFCC-shaped input resident in HBM; random-init weights",
            "config": {"workload": ("PCM -> GPU MFCC -> " if args.e2e else "")
                                   + WORKLOADS.get(args.model, f"{args.model} eval forward"),
                       "per_gpu_batch": B, "global_batch": world * B,
                       "parallelism": f"batch-shard x{world} (no data-path collective)"},
            "model_tflops": round(value * flop_clip / 1e12, 2),
            "roofline": (res_roofline(prec, cfg, kms, nlaunch, kflop, B, args.model) if is_res else
                         {"bound": "mfma",
                          "kernel": ("honk::cnn::conv_gemm_kernel<.., X3=false> (implicit-GEMM conv/linear, fp32 MFMA)"
                                     if prec == "f32" else
                                     "honk::cnn conv kernels in bf16x3 (conv1x3/conv2x3 for cnn-trad-pool2, "
                                     "else conv_gemm_kernel<.., X3=true>; 3 bf16 MFMA products per MAC; "
                                     "peak = bf16 peak / 3)"),
                          "achieved": round(achieved, 2) if achieved else None,
                          "peak": peak, "unit": "TFLOP/s",
                          "frac": round(achieved / peak, 4) if achieved else None,
                          "traffic": None,
                          "launches": nlaunch, "avg_launch_ms": round(avg_ms, 4),
                          "flop_per_launch": kflop / max(nlaunch, 1)}),
            "parity": {"top1_agreement_vs_oracle": top1, "max_abs_logit_err_vs_oracle_f64": maxerr,
                       "sample_clips": len(idx)},
        }
        res.update(alts)
        if c2 is not None:
            res["c2_cnn_trad_pool2"] = c2
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
        print(json.dumps(res), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
