"""Caching-allocator behaviour of the C3 training step: hipMalloc calls (num_device_alloc)
and reserved memory over 20 steps after 5 warm ones, per Policy override.

    python tools/alloc_probe.py [FIELD=VALUE ...]
"""
import os, sys, time
REPO = "/root/repo" if os.path.exists("/root/repo") else os.environ["GRAFT_REPO_ROOT"]
sys.path[:0] = [REPO, os.path.join(REPO, "hulk-keypoints_amd")]
import torch
from src.model import KeypointsGauss
from oracle import recipe
from hkp import train
from hkp.policy import DEFAULT
dev = torch.device("cuda", 0)
kw = {}
for item in sys.argv[1:]:
    k, _, v = item.partition("=")
    cur = getattr(DEFAULT, k)
    kw[k] = (v.lower() in ("1", "true")) if isinstance(cur, bool) else type(cur)(v)
pol = DEFAULT.with_(**kw)
B, K, H, W = 8, 4, 480, 640
m = KeypointsGauss(K, H, W, pretrained=False, policy=pol).to(dev)
x = recipe.to_tensor_nchw(recipe.seeded_images_u8(B, H, W, 1)).to(dev)
uv = torch.from_numpy(recipe.seeded_keypoints(B, K, H, W, 2)).to(dev)
t = train.Trainer(m)
for _ in range(5):
    t.step(x, uv)
torch.cuda.synchronize()
keys = ["num_device_alloc", "num_device_free", "num_alloc_retries", "num_sync_all_streams", "num_ooms"]
s0 = torch.cuda.memory_stats(dev)
t0 = time.perf_counter()
for _ in range(20):
    t.step(x, uv)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 20
s1 = torch.cuda.memory_stats(dev)
print(sys.argv[1:], "step %.2f ms" % (dt * 1e3))
for k in keys:
    print(k, s0.get(k), "->", s1.get(k))
print("reserved GB", torch.cuda.memory_reserved(dev) / 1e9)

if os.environ.get("HKP_PROBE_STEADY"):
    # the same 20-step timing once the allocator has levelled off
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(20):
            t.step(x, uv)
        torch.cuda.synchronize()
        print("steady 20 steps: %.2f ms/step, device allocs %d" % ((time.perf_counter() - t0) / 20 * 1e3,
              torch.cuda.memory_stats(dev).get("num_device_alloc")), flush=True)

if os.environ.get("HKP_PROBE_LONG"):
    # does the reserved memory level off?
    for i in range(12):
        for _ in range(10):
            t.step(x, uv)
        torch.cuda.synchronize()
        st = torch.cuda.memory_stats(dev)
        print("after %3d more steps: reserved %.1f GB, device allocs %d, allocated %.1f GB" % (
            10 * (i + 1), torch.cuda.memory_reserved(dev) / 1e9, st.get("num_device_alloc"),
            st.get("allocated_bytes.all.current", 0) / 1e9), flush=True)

if os.environ.get("HKP_PROBE_HISTORY"):
    # which call sites make the segments the steady state keeps adding
    torch.cuda.memory._record_memory_history(max_entries=200000)
    for _ in range(3):
        t.step(x, uv)
    torch.cuda.synchronize()
    snap = torch.cuda.memory._snapshot()
    from collections import Counter
    sites = Counter()
    acts = Counter(ev.get("action") for tr in snap.get("device_traces", []) for ev in tr)
    print("trace actions:", dict(acts))
    segs = [ev for tr in snap.get("device_traces", []) for ev in tr if ev.get("action") == "segment_alloc"]
    if segs:
        print("first segment_alloc frames:", [(f.get("filename"), f.get("line"), f.get("name")) for f in segs[0].get("frames", [])][:12])
    for trace in snap.get("device_traces", []):
        for ev in trace:
            if ev.get("action") == "segment_alloc":
                fr = [f for f in ev.get("frames", []) if f.get("filename", "").endswith(".py") and "torch" not in f.get("filename", "")]
                key = " <- ".join("%s:%d %s" % (os.path.basename(f["filename"]), f["line"], f["name"]) for f in fr[:3])
                sites[(key, ev.get("size"))] += 1
    for (k, sz), n in sites.most_common(25):
        print("%3d x %8.1f MB  %s" % (n, sz / 1e6, k))
