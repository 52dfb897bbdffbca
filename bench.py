#!/usr/bin/env python3
"""Benchmark of the keypoint-heatmap hot path on MI355X (BASELINE.json metric:
images/sec, 640x480, N keypoints).

Default workload = BASELINE config C2: ResNet-34-8s, K=4, 640x480, batch 32
inference per GPU (train-mode BN exactly like the reference's analysis.py /
Prediction.predict, fused K-channel head, heatmap + argmax decode).
``--mode train`` times one training iteration (forward, fp64 BCE, backward,
Adam) instead (config C3 per-GPU shard: --batch 8).

One process per GPU (torchrun for N>1); each rank owns its own batch
(weak scaling: the inference path needs no collective; training all-reduces
gradients over RCCL).  Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (REPO, os.path.join(REPO, "hulk-keypoints_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: Peak FP32 (matrix), dense
PEAK_FP16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/FP16 MFMA ~2.5 PF dense (spec)
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["infer", "train"], default="infer")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default 32 infer / 8 train)")
    ap.add_argument("--backbone", default="resnet34")
    ap.add_argument("--keypoints", type=int, default=4)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--precision", choices=["fp32", "f16x3", "f16"], default=None,
                    help="NHWC conv arithmetic (default: f16x3 = fp32-accurate split fp16 MFMA)")
    ap.add_argument("--input", choices=["f32", "u8"], default="f32",
                    help="f32: the reference's ToTensor NCHW tensor; u8: the cv2.imread-style uint8 HWC batch "
                         "(ToTensor fused into the stem, SURVEY 8(f1))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="budget for the CPU baseline sample")
    return ap.parse_args()


def conv_flops_per_image(backbone, k, H, W):
    """Algorithmic FLOPs (2*MAC) of the backbone convs + K-channel head for one image."""
    from oracle.cpu_ref import layer_plan  # plan arithmetic only (no compute)
    h, w = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    fl = 2.0 * h * w * 64 * 3 * 49
    h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    for b in layer_plan(backbone):
        s, d, cin, pl = b["stride"], b["dilation"], b["inplanes"], b["planes"]
        ho, wo = (h - 1) // s + 1, (w - 1) // s + 1
        if b["kind"] == "basic":
            fl += 2.0 * ho * wo * pl * cin * 9 + 2.0 * ho * wo * pl * pl * 9
        else:
            fl += 2.0 * h * w * pl * cin + 2.0 * ho * wo * pl * pl * 9 + 2.0 * ho * wo * pl * 4 * pl
        if b["downsample"] is not None:
            fl += 2.0 * ho * wo * b["downsample"][1] * cin
        h, w = ho, wo
    c_last = 512 * (4 if backbone == "resnet50" else 1)
    fl += 2.0 * h * w * k * c_last
    return fl


class LaunchTimer:
    """HIP-event timing of each conv launch, on the stream it is launched on
    (torch's current stream — the one libhulkkp launches on)."""

    def __init__(self):
        self.rec = []
        self.on = False

    def __call__(self, sym, flops, nbytes, launch):
        if not self.on:
            launch()
            return
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        launch()
        e.record()
        self.rec.append((sym, flops, nbytes, s, e))

    def summary(self):
        torch.cuda.synchronize()
        agg = {}
        for sym, fl, nb, s, e in self.rec:
            a = agg.setdefault(sym, [0, 0.0, 0.0, 0.0])
            a[0] += 1
            a[1] += fl
            a[2] += nb
            a[3] += s.elapsed_time(e)
        return agg


def pmc_traffic(kernel_sym, tag):
    """HBM bytes per launch of `kernel_sym` from the committed rocprofv3 PMC summary
    (profiles/*<tag>*pmc*.json, separate FETCH_SIZE / WRITE_SIZE passes):
    (FETCH_SIZE * 2 + WRITE_SIZE) * 1024 — gfx950's FETCH_SIZE counts half of a
    wide streaming read (MI355X_MICROARCH.md §HBM).  None if no summary matches."""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*%s*pmc*.json" % tag)), reverse=True):
        try:
            data = json.load(open(path))
        except (OSError, ValueError):
            continue
        for name, c in data.items():
            if kernel_sym.split("<")[0] in name and kernel_sym.split("<")[1].rstrip(">") in name.replace(" ", ""):
                if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                    return (c["FETCH_SIZE"] * 2 + c["WRITE_SIZE"]) * 1024, os.path.basename(path)
    return None, None


def cpu_baseline(args, budget_s):
    """Oracle (reference-faithful CPU restatement: 1000-ch head, train-mode BN)
    timed on this host's cores on a bounded sample of the same workload."""
    from oracle import cpu_ref, recipe
    # the host share of one GPU on the box (OMP_NUM_THREADS is set to it there)
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "16")))
    cores = torch.get_num_threads()
    sd = recipe.seeded_state_dict(args.backbone, 0)
    x = recipe.to_tensor_nchw(recipe.seeded_images_u8(1, args.height, args.width, 1234))
    with torch.no_grad():
        cpu_ref.forward(sd, x, args.backbone, args.keypoints)   # warm-up
        n, t0 = 0, time.time()
        while n < 1 or (n < 30 and time.time() - t0 < budget_s):
            h = cpu_ref.forward(sd, x, args.backbone, args.keypoints)
            cpu_ref.argmax_yx(h)
            n += 1
        dt = time.time() - t0
    return {"value": n / dt, "unit": "images/sec", "cores": cores, "kind": "port",
            "sample": "%d x batch-1 %dx%d %s-8s K=%d inference (faithful 1000-ch head, train-mode BN, argmax), "
                      "oracle/cpu_ref.py on torch CPU, %d threads" % (n, args.width, args.height, args.backbone,
                                                                      args.keypoints, cores)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.batch is None:
        args.batch = 32 if args.mode == "infer" else 8
    dist = world > 1
    if dist:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    import hkp
    from hkp import ops
    from src.model import KeypointsGauss
    from oracle import recipe  # synthetic inputs (seeded images / keypoints only)

    hkp.lib()
    from hkp import net as hkp_net
    precision = args.precision or "f16x3"
    hkp_net.set_conv_precision(precision)
    B, K, H, W = args.batch, args.keypoints, args.height, args.width
    torch.manual_seed(1234 + rank)
    model = KeypointsGauss(K, H, W, backbone=args.backbone, pretrained=False).to(dev)
    imgs = recipe.seeded_images_u8(B, H, W, 1234 + rank)
    x = recipe.to_tensor_nchw(imgs).to(dev) if args.input == "f32" else torch.from_numpy(imgs).to(dev)
    uv = torch.from_numpy(recipe.seeded_keypoints(B, K, H, W, 99 + rank)).to(dev)

    if args.mode == "infer":
        def step():
            with torch.no_grad():
                return model.heatmaps_and_keypoints(x)
    else:
        from hkp import train as hkp_train
        trainer = hkp_train.Trainer(model, lr=1e-4, weight_decay=1e-4, distributed=dist)

        def step():
            return trainer.step(x, uv)

    timer = LaunchTimer()
    ops.set_observer(timer)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = t.item()

    # roofline pass: the same steps again with every conv launch event-timed
    timer.on = True
    for _ in range(max(3, min(args.steps, 10))):
        step()
    agg = timer.summary()
    timer.on = False
    ops.set_observer(None)

    images = B * args.steps * world
    value = images / elapsed
    fl_img = conv_flops_per_image(args.backbone, K, H, W)
    if rank != 0:
        if dist:
            torch.distributed.destroy_process_group()
        return
    # dominant kernel = the conv symbol with the most event-timed time
    dom_sym, (cnt, fl, nb, ms) = max(agg.items(), key=lambda kv: kv[1][3])
    alg = (fl / cnt) / ((ms / cnt) * 1e-3) / 1e12          # algorithmic (fp32-equivalent) TFLOP/s
    if dom_sym.startswith(("conv_split_kernel", "conv_x3_kernel", "wgrad_x3_kernel")):
        passes = 3 if "_x3_" in dom_sym else int(dom_sym.split("<")[1].split(",")[2])
        achieved, peak = alg * passes, PEAK_FP16_MFMA_TFLOPS    # issued fp16 MFMA FLOPs vs dense fp16 peak
    else:
        passes, achieved, peak = 0, alg, PEAK_FP32_MFMA_TFLOPS
    all_ms = sum(v[3] for v in agg.values())
    all_fl = sum(v[1] for v in agg.values())
    dtype = {"fp32": "f32", "f16x3": "f32 (f16x3 split-precision MFMA, fp32-accurate)", "f16": "f16"}[precision]
    out = {
        "metric": "images/sec (640x480, N keypoints) inference+train at 1/2/4/8 MI355X",
        "value": value, "unit": "images/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": dtype, "data": "synthetic (seeded uint8 BGR images; random-init weights)",
        "config": {"workload": "%s %s-8s K=%d %dx%d batch %d/GPU (%s)" % (
            "inference (C2)" if args.mode == "infer" else "training step (C3 shard)", args.backbone, K, W, H, B,
            "train-mode BN, fused K-ch head, heatmap + argmax" if args.mode == "infer"
            else "BCE fp64, Adam lr1e-4 wd1e-4"),
            "mode": args.mode, "backbone": args.backbone, "keypoints": K, "height": H, "width": W,
            "batch_per_gpu": B, "global_batch": B * world, "parallelism": "dp%d" % world,
            "input": "fp32 NCHW (ToTensor)" if args.input == "f32" else "uint8 HWC BGR (ToTensor fused into the stem)"},
        "roofline": {"bound": "mfma", "kernel": dom_sym, "achieved": achieved, "peak": peak,
                     "unit": "TFLOP/s", "frac": achieved / peak, "traffic": None,
                     "fp32_equivalent_tflops": alg, "frac_of_fp32_mfma_peak": alg / PEAK_FP32_MFMA_TFLOPS,
                     "mfma_passes_per_fp32_mac": passes or 1,
                     "launches_per_step": cnt // max(3, min(args.steps, 10)),
                     "avg_launch_ms": ms / cnt, "algorithmic_gflop_per_launch": fl / cnt / 1e9,
                     "all_convs_tflops": all_fl / (all_ms * 1e-3) / 1e12,
                     "conv_share_of_step": (all_ms / max(3, min(args.steps, 10))) / (elapsed / args.steps * 1e3)},
        "model_tflops": value / world * fl_img * (3 if args.mode == "train" else 1) / 1e12,
        "peak_hbm_gb": torch.cuda.max_memory_allocated(dev) / 1e9,
    }
    tag = "infer_c2" if args.mode == "infer" else "train_c3"
    traffic, src = pmc_traffic(dom_sym.replace(" ", ""), tag) if (args.backbone, K, H, W) == ("resnet34", 4, 480,
                                                                                             640) else (None, None)
    out["roofline"]["traffic"] = traffic
    out["roofline"]["traffic_source"] = src
    out["roofline"]["algorithmic_bytes_per_launch"] = nb / cnt
    if not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
    print(json.dumps(out))
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
