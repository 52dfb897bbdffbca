#!/usr/bin/env python3
"""Benchmark of the keypoint-heatmap hot path on MI355X (BASELINE.json metric:
images/sec, 640x480, N keypoints, inference+train).

Default workload = BASELINE config C2: ResNet-34-8s, K=4, 640x480, batch 32
inference per GPU (train-mode BN exactly like the reference's analysis.py /
Prediction.predict, fused K-channel head, heatmap + argmax decode) — the
line's `value`.  The same run also times, as extra keys of the one JSON line:
  * "train": one training iteration per step (forward, fused fp64 BCE,
    backward, RCCL all-reduce of gradients at N>1, FusedAdam) on config C3's
    per-GPU shard (batch 8 of the 64-image global batch at N=8);
  * "fp32_exact": C2 with exact-fp32 MFMA convs (--precision fp32) beside the
    default f16x3 split arithmetic;
  * "cpu_baseline": the oracle (reference-faithful CPU restatement) on this
    host's cores: C2 inference at batch 1 and 4 and the C1 training step.
``--mode train`` makes the training step the main line instead.

One process per GPU.  ``--gpus N`` without a torchrun environment relaunches
itself under ``torch.distributed.run`` as a child process (before any GPU
call); under torchrun N must equal WORLD_SIZE.  Inference shards by image
(weak scaling): each rank runs its own batch and the int32 keypoints are
all-gathered each step (hkp.parallel); training all-reduces gradients over RCCL.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (REPO, os.path.join(REPO, "hulk-keypoints_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: Peak FP32 (matrix), dense
PEAK_FP16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/FP16 MFMA ~2.5 PF dense (spec)
PEAK_HBM_GBPS = 8000.0          # MI355X_MICROARCH.md: HBM3E ~8 TB/s
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["infer", "train"], default="infer")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default 32 infer / 8 train)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="strong scaling: the job's batch, split over the N ranks (per-rank batch = G/N; rank r "
                         "takes images [r*G/N, (r+1)*G/N) of the seeded G-image batch)")
    ap.add_argument("--backbone", default="resnet34")
    ap.add_argument("--keypoints", type=int, default=4)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--precision", choices=["fp32", "f16x3", "f16", "f16x2w", "f16x2a"], default=None,
                    help="NHWC conv arithmetic (default: f16x3 = fp32-accurate split fp16 MFMA)")
    ap.add_argument("--input", choices=["f32", "u8"], default="f32",
                    help="f32: the reference's ToTensor NCHW tensor; u8: the cv2.imread-style uint8 HWC batch "
                         "(ToTensor fused into the stem, SURVEY 8(f1))")
    ap.add_argument("--sync-bn", action="store_true",
                    help="N>1: BN statistics (and, training, their backward sums) over the global batch")
    ap.add_argument("--stage-precision", default=None, metavar="L1,L2,L3,L4",
                    help="inference with --precision f16: per-stage conv arithmetic, each of f16 / f16x3 for "
                         "layer1..layer4 (Policy.stage_precision; DESIGN 'Per-stage precision')")
    ap.add_argument("--no-extras", action="store_true", help="main line only (no train / fp32 legs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="budget for the CPU baseline sample")
    ap.add_argument("--tune", action="append", default=[], metavar="FIELD=VALUE",
                    help="A/B tooling: a non-default tuning field of hkp.policy.Policy (repeatable)")
    ap.add_argument("--lib", default=None, help="A/B tooling: load this build of libhulkkp.so instead")
    ap.add_argument("--rehearse-gloo", action="store_true",
                    help="N>1 on a one-GPU box: ranks share the GPU over gloo (rehearses the multi-rank path; "
                         "never a measurement — RCCL refuses two ranks on one device)")
    return ap.parse_args()


def tuning(args):
    """--tune FIELD=VALUE pairs → Policy keyword arguments (typed like the defaults)."""
    from hkp.policy import DEFAULT, TUNING_FIELDS
    kw = {}
    for item in args.tune:
        k, _, v = item.partition("=")
        if k not in TUNING_FIELDS:
            raise SystemExit("bench.py: --tune %s: not a tuning field (%s)" % (k, ", ".join(TUNING_FIELDS)))
        cur = getattr(DEFAULT, k)
        kw[k] = (v.lower() in ("1", "true", "yes")) if isinstance(cur, bool) else type(cur)(v)
    return kw


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def relaunch_distributed(n):
    """bench.py --gpus N outside torchrun: run N ranks under torch.distributed.run
    as a child process (this process has not touched the GPU) and return its exit
    code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def conv_flops_per_image(backbone, k, H, W):
    """Algorithmic FLOPs (2*MAC) of the backbone convs + K-channel head for one image."""
    from oracle.cpu_ref import layer_plan  # plan arithmetic only (no compute)
    h, w = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
    fl = 2.0 * h * w * 64 * 3 * 49
    h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    for b in layer_plan(backbone):
        s, cin, pl = b["stride"], b["inplanes"], b["planes"]
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
    (torch's current stream — the one libhulkkp launches on; the side stream
    for an overlapped wgrad)."""

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


def _nospace(s):
    return s.replace(" ", "")


def _tail_of(kernel_sym):
    """The split-K tail kernel a 256x256 one-tile conv launch ends in (its last,
    partly filled round), as a rocprof name fragment, or None."""
    if not kernel_sym.startswith(("conv_x3_kernel<256,", "conv_x3_a3_kernel<")):
        return None
    p = _nospace(kernel_sym).rstrip(">").split(",")[-1].split("<")[-1]      # the operand layout P
    return "::conv_x3_tail_kernel<256,%s>(" % p


def pmc_traffic(kernel_sym, tag):
    """HBM bytes per launch of `kernel_sym` from the newest committed rocprofv3 PMC
    summary (profiles/*<tag>*pmc*.json, separate FETCH_SIZE / WRITE_SIZE passes):
    (FETCH_SIZE * 2 + WRITE_SIZE) * 1024 — gfx950's FETCH_SIZE counts half of a
    wide streaming read (MI355X_MICROARCH.md §HBM).  The kernel name must match
    exactly (spaces ignored).  A 256x256 conv_x3 launch whose last round runs as
    the split-K tail (conv_x3_tail_kernel, same stream, inside the same event
    pair) gets the tail's bytes and time folded in per main dispatch, so the
    figures describe what the event timed.  Returns (bytes, source file, the PMC
    pass's average ms of the same scope — serialised kernels, reported as
    pmc_pass_avg_ms, not as the launch time — folded kernel or None); Nones if
    no summary has the kernel."""
    import glob
    want = "::" + _nospace(kernel_sym) + "("
    tail_want = _tail_of(kernel_sym)
    paths = glob.glob(os.path.join(REPO, "profiles", "*%s*pmc*.json" % tag))
    for path in sorted(paths, reverse=True):       # rNN_..._vNN names: newest round / version first
        try:
            data = json.load(open(path))
        except (OSError, ValueError):
            continue
        for name, c in data.items():
            if want in _nospace(name) and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                nbytes = (c["FETCH_SIZE"] * 2 + c["WRITE_SIZE"]) * 1024
                ms = c.get("avg_duration_ns", 0.0) * 1e-6
                folded = None
                for tname, t in data.items():
                    if tail_want and tail_want in _nospace(tname) and "FETCH_SIZE" in t and "WRITE_SIZE" in t:
                        per = t.get("dispatches", 0) / max(c.get("dispatches", 1), 1)
                        nbytes += (t["FETCH_SIZE"] * 2 + t["WRITE_SIZE"]) * 1024 * per
                        ms += t.get("avg_duration_ns", 0.0) * 1e-6 * per
                        folded = tname
                return nbytes, os.path.basename(path), ms or None, folded
    return None, None, None, None


def trace_avg_ms(kernel_sym, tag):
    """Average duration of `kernel_sym` from the newest committed rocprofv3
    --kernel-trace --stats summary (profiles/*<tag>*kernel_stats*.csv), the same
    scope the HIP events time: a 256x256 conv_x3 launch's split-K tail
    (conv_x3_tail_kernel) folded in per main dispatch.  The PMC passes serialise
    kernels and run at a different clock, so their durations are not used for
    this.  Returns (ms, source file) or (None, None)."""
    import csv
    import glob
    want = "::" + _nospace(kernel_sym) + "("
    tail_want = _tail_of(kernel_sym)
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*%s*kernel_stats*.csv" % tag)), reverse=True):
        try:
            rows = list(csv.DictReader(open(path)))
        except (OSError, ValueError):
            continue
        main = [r for r in rows if want in _nospace(r["Name"])]
        if not main:
            continue
        calls, tot = int(main[0]["Calls"]), float(main[0]["TotalDurationNs"])
        for r in rows:
            if tail_want and tail_want in _nospace(r["Name"]):
                tot += float(r["TotalDurationNs"])
        return tot / calls * 1e-6, os.path.basename(path)
    return None, None


def host_cores():
    """CPUs this process may use: os.cpu_count(), narrowed by the affinity mask and
    the cgroup CPU quota (a GPU box shows the whole machine's CPUs in
    os.cpu_count() but grants one GPU's share)."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, budget_s):
    """Oracle (reference-faithful CPU restatement: 1000-ch head, train-mode BN,
    fp64 BCE, Adam) timed on this host's cores on a bounded sample: C2-shape
    inference at batch 1 and 4, and the C1 training step (R18-8s K=2 320x240
    batch 4, train.py:32-36).  One warm-up each, then the median of up to 3."""
    import statistics

    from oracle import cpu_ref, recipe
    cores = host_cores()
    torch.set_num_threads(cores)
    sd = recipe.seeded_state_dict(args.backbone, 0)

    def timed(fn, reps):                   # each of the three legs gets a third of the budget
        t_start = time.time()
        fn()
        ts = []
        for _ in range(reps):
            if ts and time.time() - t_start > budget_s / 3:
                break
            t0 = time.time()
            fn()
            ts.append(time.time() - t0)
        return statistics.median(ts), len(ts)

    legs = {}
    with torch.no_grad():
        for b in (1, 4):
            x = recipe.to_tensor_nchw(recipe.seeded_images_u8(b, args.height, args.width, 1234))

            def infer():
                cpu_ref.argmax_yx(cpu_ref.forward({k: v.clone() for k, v in sd.items()}, x, args.backbone,
                                                  args.keypoints))
            t, n = timed(infer, 3)
            legs["infer_b%d" % b] = {"images_per_sec": b / t, "ms_per_batch": t * 1e3, "samples": n}
    c1 = dict(backbone="resnet18", k=2, H=240, W=320, B=4)
    sd1 = recipe.seeded_state_dict(c1["backbone"], 0)
    x1 = recipe.to_tensor_nchw(recipe.seeded_images_u8(c1["B"], c1["H"], c1["W"], 4321))
    uv1 = recipe.seeded_keypoints(c1["B"], c1["k"], c1["H"], c1["W"], 99)
    trainer = cpu_ref.OracleTrainer(sd1, c1["backbone"], c1["k"])
    t, n = timed(lambda: trainer.step(x1, uv1), 3)
    legs["train_c1"] = {"images_per_sec": c1["B"] / t, "ms_per_step": t * 1e3, "samples": n,
                        "workload": "C1: R18-8s K=2 320x240 batch 4 train step (BCE fp64 + Adam)"}
    return {"value": legs["infer_b4"]["images_per_sec"], "unit": "images/sec", "cores": cores, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(),
            "sample": "oracle/cpu_ref.py on torch CPU, %d threads; value = %dx%d %s-8s K=%d inference at batch 4 "
                      "(faithful 1000-ch head, train-mode BN, argmax); also batch 1 and the C1 train step"
                      % (cores, args.width, args.height, args.backbone, args.keypoints),
            "legs": legs}


def workload_name(mode, backbone, k, h, w, precision, batch, global_batch=None, world=1):
    """The BASELINE.json config a bench line measures (C2..C5; C3/C5 per-GPU shards of
    their DP jobs; north_star's strong-scaling batch-64 C2 inference), or "custom"
    with its shape."""
    shape = (mode, backbone, k, w, h)
    fp32_class = precision in ("fp32", "f16x3")
    if global_batch:
        if shape == ("infer", "resnet34", 4, 640, 480) and global_batch == NORTH_STAR_GLOBAL_BATCH and fp32_class:
            return "north_star scaling: C2 batch %d over %d GPU(s)" % (global_batch, world)
        return "custom strong-scaling %s (global batch %d)" % ("inference" if mode == "infer" else "training",
                                                               global_batch)
    if shape == ("infer", "resnet34", 4, 640, 480) and batch == 32 and fp32_class:
        return "C2 inference"
    if shape == ("train", "resnet34", 4, 640, 480) and batch == 8:
        return "C3 shard (batch 64 over 8 GPUs) training step"
    if shape == ("infer", "resnet50", 8, 640, 480) and batch == 128 and precision == "f16":
        return "C4 fp16 inference"
    if shape == ("train", "resnet50", 8, 1280, 960) and batch == 32:
        return "C5 shard (batch 256 over 8 GPUs) training step"
    if shape == ("train", "resnet18", 2, 320, 240) and batch == 4:
        return "C1 training step"
    return "custom %s" % ("inference" if mode == "infer" else "training step")


NORTH_STAR_GLOBAL_BATCH = 64      # north_star: ">=6x ... 1->8 GPUs on 640x480 batch-64 inference"


def north_star_leg(precision, args, dev, rank, world):
    """north_star's scaling workload: C2 inference (R34-8s K=4 640x480) on a 64-image
    batch split over the ranks (strong scaling; rank r takes images [r*64/N,
    (r+1)*64/N) of the seeded batch; train-mode BN per rank = a per-shard run of the
    reference).  On one GPU it also times the 8-image shard the batch puts
    on each rank at N = 8, whose rate bounds the 1 -> 8 speedup from compute:
    8 * img/s(B=8) / img/s(B=64) (the all-gather of 2 KB of keypoints aside)."""
    G = NORTH_STAR_GLOBAL_BATCH
    leg = run_leg("infer", precision, G // world, args, dev, rank, world, args.steps, args.warmup,
                  shard_of=(G, rank))
    leg["workload"] = "north_star scaling: C2 batch %d over %d GPU(s) (R34-8s K=4 640x480, %d images per rank, " \
                      "per-rank train-mode BN, keypoints all-gathered at N>1)" % (G, world, G // world)
    leg["scaling"] = "strong"
    if world == 1:
        b8 = run_leg("infer", precision, G // 8, args, dev, rank, 1, args.steps, args.warmup, shard_of=(G, 7))
        leg["shard_b8"] = {"value": b8["value"], "ms_per_step": b8["ms_per_step"],
                           "images": "images 56-63 of the seeded 64-image batch (rank 7's shard at N = 8)",
                           "dominant_kernel": b8["roofline"]["kernel"], "frac": b8["roofline"]["frac"]}
        leg["predicted_speedup_1to8_compute_ceiling"] = 8.0 * b8["value"] / leg["value"]
    return leg


def run_leg(mode, precision, batch, args, dev, rank, world, steps, warmup, shard_of=None):
    """Time `steps` steps of one workload; return its metrics (rank 0 gets them).
    shard_of = (G, i): the images are slice i (batch images) of the seeded G-image
    batch (a strong-scaling shard); default: each rank's own seeded batch."""
    import hkp
    from hkp import ops, parallel
    from hkp.policy import Policy
    from oracle import recipe  # synthetic inputs (seeded images / keypoints only)
    from src.model import KeypointsGauss

    hkp.lib()
    dist = world > 1
    sync_bn = dist and getattr(args, "sync_bn", False)
    B, K, H, W = batch, args.keypoints, args.height, args.width
    # a strong-scaling shard (shard_of) is a slice of ONE job: every rank runs the same
    # random-init model; weak scaling gives each rank its own seed
    torch.manual_seed(1234 if shard_of is not None else 1234 + rank)
    stage = tuple(args.stage_precision.split(",")) if getattr(args, "stage_precision", None) else ()
    pol = Policy(precision=precision, stage_precision=stage if mode == "infer" and precision == "f16" else (),
                 **tuning(args))
    model = KeypointsGauss(K, H, W, backbone=args.backbone, pretrained=False, policy=pol).to(dev)
    if shard_of is not None:
        G, i = shard_of
        imgs = recipe.seeded_images_u8(G, H, W, 1234)[i * B:(i + 1) * B]
    else:
        imgs = recipe.seeded_images_u8(B, H, W, 1234 + rank)
    x = recipe.to_tensor_nchw(imgs).to(dev) if args.input == "f32" else torch.from_numpy(imgs).to(dev)
    uv = torch.from_numpy(recipe.seeded_keypoints(B, K, H, W, 99 + rank)).to(dev)

    if mode == "infer":
        gathered = torch.empty((world * B, K, 2), device=dev, dtype=torch.int32) if dist else None
        if sync_bn:
            model.policy = model.policy.with_(sync_bn=True)

        def step():
            with torch.no_grad():
                hm, yx = model.heatmaps_and_keypoints(x)
                if dist:                                   # every rank ends with all keypoints
                    parallel.gather_keypoints_fixed(yx, gathered)
                return hm
    else:
        from hkp import train as hkp_train
        trainer = hkp_train.Trainer(model, lr=1e-4, weight_decay=1e-4, distributed=dist, sync_bn=sync_bn)

        def step():      # (SyncBN: equal shards of the global batch, no per-step host collective)
            return trainer.step(x, uv, global_batch=B * world if sync_bn else None)

    timer = LaunchTimer()
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
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
    reps = max(3, min(steps, 10))
    ops.set_observer(timer)          # not before: the timed steps carry no instrumentation
    timer.on = True
    for _ in range(reps):
        step()
    agg = timer.summary()
    timer.on = False
    ops.set_observer(None)
    peak_mem = torch.cuda.max_memory_allocated(dev) / 1e9
    del model, x, uv
    if mode != "infer":
        del trainer
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)

    value = B * steps * world / elapsed
    fl_img = conv_flops_per_image(args.backbone, K, H, W)
    # dominant kernel = the conv symbol with the most event-timed time
    dom_sym, (cnt, fl, nb, ms) = max(agg.items(), key=lambda kv: kv[1][3])
    alg = (fl / cnt) / ((ms / cnt) * 1e-3) / 1e12          # algorithmic (fp32-equivalent) TFLOP/s
    if dom_sym.startswith(("conv_x3_kernel", "conv_x3_a3_", "conv_x3_halo_kernel", "wgrad_x3_kernel")):
        # the x3 LDS-DMA kernels: fp16 MFMAs per fp32 MAC — 3 (f16x3), 2 (f16x2w / f16x2a: two of
        # the three products), 1 (f16)
        passes = {"f16x3": 3, "f16x2w": 2, "f16x2a": 2}.get(precision, 1)
        achieved, peak = alg * passes, PEAK_FP16_MFMA_TFLOPS    # issued fp16 MFMA FLOPs vs dense fp16 peak
    else:
        passes, achieved, peak = 1, alg, PEAK_FP32_MFMA_TFLOPS
    all_ms = sum(v[3] for v in agg.values())
    all_fl = sum(v[1] for v in agg.values())
    roof = {"bound": "mfma", "kernel": dom_sym, "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
            "frac": achieved / peak, "traffic": None,
            "fp32_equivalent_tflops": alg, "mfma_passes_per_fp32_mac": passes,
            "launches_per_step": cnt // reps, "avg_launch_ms": ms / cnt,
            "algorithmic_gflop_per_launch": fl / cnt / 1e9,
            "algorithmic_bytes_per_launch": nb / cnt,
            "all_convs_tflops": all_fl / (all_ms * 1e-3) / 1e12,
            "conv_share_of_step": (all_ms / reps) / (elapsed / steps * 1e3)}
    if passes == 3:
        # f16x3 issues 3 fp16 MFMAs per fp32 MAC: its own ceiling is a third of the fp16 peak
        roof["frac_of_x3_ceiling"] = alg / (PEAK_FP16_MFMA_TFLOPS / 3)
    # the classic roofline per launch: attainable time = max(issued FLOPs / MFMA
    # peak, algorithmic bytes / HBM peak); frac_of_roofline = sum attainable /
    # sum measured over the dominant symbol's launches (= frac when every launch
    # is MFMA-bound; short-K 1x1 GEMMs writing wide fp16 outputs are HBM-bound)
    t_att = t_meas = t_hbm = 0.0
    for sym, f, b, s_ev, e_ev in timer.rec:
        if sym != dom_sym:
            continue
        tc, tm = f * passes / (peak * 1e12), b / (PEAK_HBM_GBPS * 1e9)
        t_att += max(tc, tm)
        t_meas += s_ev.elapsed_time(e_ev) * 1e-3
        t_hbm += tm if tm > tc else 0.0
    if t_meas > 0:
        roof["frac_of_roofline"] = t_att / t_meas
        roof["hbm_bound_share_of_attainable"] = t_hbm / t_att if t_att > 0 else 0.0
    # the committed profiles of this exact workload (batch included: a trace's average
    # launch time belongs to its own launch sizes)
    r34 = (args.backbone, K, H, W) == ("resnet34", 4, 480, 640) and precision == "f16x3"
    c4 = (args.backbone, K, H, W) == ("resnet50", 8, 480, 640) and precision == "f16" and mode == "infer" and B == 128 \
        and not args.stage_precision
    c5 = (args.backbone, K, H, W) == ("resnet50", 8, 960, 1280) and precision == "f16x3" and mode == "train" \
        and B == 32
    tag = None
    if r34:
        tag = {("infer", 32): "infer_c2", ("infer", 8): "b8", ("train", 8): "train_c3"}.get((mode, B))
    if c4:
        tag = "infer_c4"
    if c5:
        tag = "train_c5"
    if tag is not None:
        (roof["traffic"], roof["traffic_source"], roof["pmc_pass_avg_ms"],
         roof["folded_kernel"]) = pmc_traffic(dom_sym, tag)
        # the kernel trace of the bench command itself (not the serialised PMC pass)
        roof["rocprof_avg_ms"], roof["rocprof_source"] = trace_avg_ms(dom_sym, tag)
    if roof["conv_share_of_step"] > 1.0:
        # training: the event pairs of the side-stream wgrads bracket time in which
        # the main stream's dgrad shares the CUs, so the conv events add up to more
        # than the step and `frac` prices shared CU time as exclusive
        roof["timing"] = "overlapped (side-stream wgrad events share CUs with the main stream)"
    if roof.get("rocprof_avg_ms"):
        # the line reproduces from profiles/: `achieved` / `frac` use the committed
        # rocprofv3 kernel trace's average duration of this symbol; the HIP-event
        # figures of this run stay beside them
        roof["achieved_events"], roof["frac_events"] = roof["achieved"], roof["frac"]
        roof["achieved"] = (fl / cnt) * passes / (roof["rocprof_avg_ms"] * 1e-3) / 1e12
        roof["frac"] = roof["achieved"] / peak
        roof["frac_from_trace"] = roof["frac"]
        roof["frac_source"] = "rocprof trace (%s); frac_events: this run's HIP events" % roof["rocprof_source"]
    return {"value": value, "ms_per_step": elapsed / steps * 1e3, "steps": steps, "warmup": warmup,
            "batch_per_gpu": B, "global_batch": B * world, "roofline": roof,
            "model_tflops": value / world * fl_img * (3 if mode == "train" else 1) / 1e12,
            "peak_hbm_gb": peak_mem}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch_distributed(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        print("bench.py: --gpus %d but WORLD_SIZE=%d (launch with torchrun --nproc-per-node %d, or without "
              "torchrun to let bench.py start the ranks)" % (args.gpus, world, args.gpus), file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    # --rehearse-gloo: N ranks share the visible GPU(s) over gloo — rehearses the
    # multi-rank path (relaunch, barriers, max-over-ranks timing, DP wiring) on a
    # one-GPU box; RCCL refuses two ranks on one device.  Never a measurement.
    rehearse = dist and args.rehearse_gloo
    if args.lib:
        from hkp import _lib
        _lib.use_library(os.path.abspath(args.lib))
    if rehearse:
        local = local % max(1, torch.cuda.device_count())
    if dist:
        torch.cuda.set_device(local)
        if rehearse:
            torch.distributed.init_process_group("gloo")
        else:
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    precision = args.precision or "f16x3"
    shard = None
    if args.global_batch:
        if args.global_batch % world or args.batch:
            print("bench.py: --global-batch %d must split evenly over %d rank(s) and excludes --batch"
                  % (args.global_batch, world), file=sys.stderr)
            sys.exit(2)
        batch, shard = args.global_batch // world, (args.global_batch, rank)
    else:
        batch = args.batch or (32 if args.mode == "infer" else 8)

    main_leg = run_leg(args.mode, precision, batch, args, dev, rank, world, args.steps, args.warmup, shard_of=shard)
    extras = {}
    default_c2 = (args.mode, args.backbone, args.keypoints, args.height, args.width) == \
        ("infer", "resnet34", 4, 480, 640)
    if not args.no_extras and default_c2 and not args.global_batch and NORTH_STAR_GLOBAL_BATCH % world == 0:
        extras["north_star_scaling"] = north_star_leg(precision, args, dev, rank, world)
    if not args.no_extras and default_c2 and not args.global_batch:
        extras["train"] = run_leg("train", precision, 8, args, dev, rank, world, args.steps, args.warmup)
        extras["train"]["workload"] = "training step (C3 shard) resnet34-8s K=4 640x480 batch 8/GPU " \
                                      "(BCE fp64, backward, RCCL grad all-reduce at N>1, FusedAdam lr1e-4 wd1e-4)"
        if precision != "fp32":
            extras["fp32_exact"] = run_leg("infer", "fp32", batch, args, dev, rank, world, max(3, args.steps // 4),
                                           2)
            extras["fp32_exact"]["workload"] = "C2 with exact-fp32 MFMA convs (v_mfma_f32_32x32x2_f32)"
    if rank != 0:
        if dist:
            torch.distributed.destroy_process_group()
        return
    if args.stage_precision and precision != "f16":
        raise SystemExit("bench.py: --stage-precision plans the plain-fp16 network (--precision f16)")
    dtype = {"fp32": "f32", "f16x3": "f32 (f16x3 split-precision MFMA, fp32-accurate)", "f16": "f16",
             "f16x2w": "f32 activations x f16 weights (2 fp16 MFMA products)",
             "f16x2a": "f16-rounded activations x split weights (2 fp16 MFMA products)"}[precision]
    B = batch
    out = {
        "metric": "images/sec (640x480, N keypoints) inference+train at 1/2/4/8 MI355X",
        "value": main_leg["value"], "unit": "images/sec", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": main_leg["ms_per_step"], "higher_is_better": True,
        "scaling": "strong" if args.global_batch else "weak",
        "vs_baseline": None, "dtype": dtype, "data": "synthetic (seeded uint8 BGR images; random-init weights)",
        "config": {"workload": "%s: %s-8s K=%d %dx%d %s batch %d/GPU (%s)" % (
            workload_name(args.mode, args.backbone, args.keypoints, args.height, args.width,
                          "f16+f16x3 stages" if args.stage_precision else precision, B, args.global_batch, world),
            args.backbone, args.keypoints, args.width, args.height,
            precision + (" (stages %s)" % args.stage_precision if args.stage_precision else ""),
            B, "train-mode BN, fused K-ch head, heatmap + argmax, keypoints all-gathered at N>1"
            if args.mode == "infer" else "BCE fp64, Adam lr1e-4 wd1e-4"),
            "mode": args.mode, "backbone": args.backbone, "keypoints": args.keypoints, "height": args.height,
            "width": args.width, "batch_per_gpu": B, "global_batch": B * world, "parallelism": "dp%d" % world,
            "bn": "sync (global-batch statistics)" if args.sync_bn and world > 1 else "per-rank",
            "collectives": ("gloo REHEARSAL (ranks share one GPU: not a measurement)" if rehearse
                            else "rccl" if world > 1 else "none"),
            "input": "fp32 NCHW (ToTensor)" if args.input == "f32" else "uint8 HWC BGR (ToTensor fused into the stem)"},
        "roofline": main_leg["roofline"],
        "model_tflops": main_leg["model_tflops"],
        "peak_hbm_gb": main_leg["peak_hbm_gb"],
    }
    out.update(extras)
    if not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
    print(json.dumps(out))
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
