"""The C5 frame (512x512, bench.c5_bench) split into stages, bf16 vs fp8 (LayerNorm fold),
each captured and replayed as a graph (round 6): encoder; pair decode (two model chains);
mono decode; the pair heads (split) — where the fp8 path does and does not pay."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from monst3r_slam_amd import model as Mdl  # noqa: E402

dev = torch.device("cuda:0")
m, _ = Mdl.build(dev)
g = torch.Generator(device=dev).manual_seed(55)
img = torch.rand(1, 3, 512, 512, device=dev, generator=g) * 2 - 1
img_k = torch.rand(1, 3, 512, 512, device=dev, generator=g) * 2 - 1
gh = gw = 32
for mode in ("bf16", "fp8"):
    m.set_fp8(mode == "fp8")
    feat_k = m.encode(img_k)[0].clone()
    st = {}
    st["f"], st["pos"] = m.encode(img)
    st["f"] = st["f"].clone()
    st["hooks"] = m.decode(st["f"][0], feat_k[0], st["pos"], gh, gw)

    def enc():
        m.encode(img)

    def dec():
        m.decode(st["f"][0], feat_k[0], st["pos"], gh, gw)

    def mono():
        m.mono(st["f"], 512, 512)

    def heads():
        m.heads(st["hooks"], gh, gw, 512, 512, split=True)
        m.join()
    out = []
    for name, fn in (("encoder", enc), ("pair decode", dec), ("mono decode+heads", mono),
                     ("pair heads", heads)):
        fn()
        torch.cuda.synchronize()
        gph = bench.capture(fn, dev)
        out.append(f"{name} {bench.time_replays(gph, dev, 20):.3f} ms")
        del gph
    print(mode + ": " + " | ".join(out), flush=True)
m.set_fp8(False)
