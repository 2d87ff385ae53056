"""The bench's timed C3 step alone, for rocprofv3 (kernel trace / PMC passes): the same
model, sequence, prefetching FramePipeline and the period's graphs as bench.py, replayed
`--steps` frames from the INIT keyframe.  The replays are bracketed by two marker launches
(m3s_retr_rownorm on one row: a kernel the step never runs), so a profile's dispatches
strictly between the two rownorm_kernel dispatches are exactly those steps.

  rocprofv3 --kernel-trace --stats -d gpurun_out/p -o step -- python tools/step_prof.py
  rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU GRBM_GUI_ACTIVE -d ... -- python ...
then tools/step_pmc_report.py summarises per step."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def marker(lib, buf, dev):
    from monst3r_slam_amd import _lib
    _lib.check(lib.m3s_retr_rownorm(_lib.ptr(buf), 1, 64, 1, _lib.ptr(buf[64:]),
                                    _lib.stream(dev)), "marker")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--out", default=None, help="JSON with the untraced-equivalent wall time")
    ap.add_argument("--group", type=int, default=2, help="frames per prefetched encoder batch")
    args = ap.parse_args()
    from monst3r_slam_amd import _lib
    from monst3r_slam_amd import sequence as S
    from monst3r_slam_amd.frontend import FramePipeline
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model, tr, seq = bench.setup(dev, 0, max(bench.SEQ_FRAMES, args.steps) + 1)
    model.serial = True
    tr.split_heads = True
    pipe = FramePipeline(tr, (bench.H, bench.W), 0, group=args.group)
    loop = S.SequenceLoop(tr, seq, pipe)
    loop.reset(parity=0)
    for w in range(args.warmup):
        loop.step(w)
    torch.cuda.synchronize(dev)
    graphs = [bench.capture(lambda k=k: loop.step(k), dev) for k in range(pipe.period)]
    lib = _lib.load()
    mbuf = torch.ones(128, dtype=torch.float32, device=dev)
    loop.reset(parity=0)
    torch.cuda.synchronize(dev)
    marker(lib, mbuf, dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        graphs[i % len(graphs)].replay()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    marker(lib, mbuf, dev)
    torch.cuda.synchronize(dev)
    res = {"steps": args.steps, "ms_per_step": el / args.steps * 1e3}
    print(json.dumps(res), flush=True)
    if args.out:
        json.dump(res, open(args.out, "w"))


if __name__ == "__main__":
    main()
