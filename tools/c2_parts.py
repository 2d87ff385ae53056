"""C2 (one 384x512 pair inference) split into its stages, each captured and replayed as a
graph (round 6): encoder alone; encoder + both decoders; the full pair with split heads;
and the heads alone on precomputed hooks — where the pair's latency goes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from monst3r_slam_amd import model as Mdl  # noqa: E402

dev = torch.device("cuda:0")
m, _ = Mdl.build(dev)
g = torch.Generator(device=dev).manual_seed(1)
img = torch.rand(1, 3, 384, 512, device=dev, generator=g) * 2 - 1
feat_k = m.encode(torch.rand(1, 3, 384, 512, device=dev, generator=g) * 2 - 1)[0].clone()
gh, gw = 24, 32
state = {}


def enc():
    state["f"], state["pos"] = m.encode(img)


def enc_dec():
    enc()
    state["hooks"] = m.decode(state["f"][0], feat_k.reshape(-1, 1024), state["pos"], gh, gw)


def full():
    m.pair(img, feat_j=feat_k, split_heads=True)
    m.join()


def heads_only():
    m.heads(state["hooks"], gh, gw, 384, 512, split=True)
    m.join()


def heads_serial():
    m.heads(state["hooks"], gh, gw, 384, 512, split=False)


res = {}
for name, fn in (("encoder", enc), ("encoder+decoders", enc_dec), ("pair (split heads)", full),
                 ("heads only (split)", heads_only), ("heads only (one stream)", heads_serial)):
    fn()
    torch.cuda.synchronize()
    gph = bench.capture(fn, dev)
    res[name] = bench.time_replays(gph, dev, 30)
    del gph
    print(f"{name:28s} {res[name]:.3f} ms", flush=True)
