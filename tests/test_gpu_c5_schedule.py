"""C5 frame schedule (bench.c5_bench): the mono branch (MonST3R self-pair decode + heads,
ego flow, flow-error mask) on side stream 1 beside the pair branch (pair decode + four
heads) — the two share only the encoder features — gives the same masked outputs, mask and
mono pointmap as running them one after the other, bit for bit, in bf16 and fp8 mode."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_c5_mono_branch_concurrent_equals_sequential(dev):
    from monst3r_slam_amd import model as Mdl
    from monst3r_slam_amd import monst3r_utils as U
    from monst3r_slam_amd import synthetic as syn
    m, _ = Mdl.build(dev)
    H5 = W5 = 512
    gh = gw = 32
    g = torch.Generator(device=dev).manual_seed(55)
    img = torch.rand(1, 3, H5, W5, device=dev, generator=g) * 2 - 1
    img_k = torch.rand(1, 3, H5, W5, device=dev, generator=g) * 2 - 1
    K = torch.from_numpy(syn.intrinsics(H5, W5)).to(dev)
    Ti = torch.tensor([0.05, 0.0, 0.01, 0, 0, 0, 1, 1.0], device=dev)
    Tk = torch.tensor([0.0, 0.0, 0.0, 0, 0, 0, 1, 1.0], device=dev)
    flow = torch.randn(2, H5, W5, device=dev, generator=g)
    for fp8 in (False, True):
        m.set_fp8(fp8)
        feat_k = m.encode(img_k)[0].clone()
        outs = []
        for conc in (False, True):
            feat_i, pos = m.encode(img)
            main = torch.cuda.current_stream(dev)
            s = m.side[1] if conc else main
            if conc:
                s.wait_stream(main)
            with torch.cuda.stream(s):
                Xm, _ = m.mono(feat_i, H5, W5)
                sR, t = U.sim3_relative_matrix(Ti, Tk)
                ego = U.ego_flow(Xm[0], sR, t, K, K)
                mask = U.dynamic_mask_from_flow(flow, ego, 0.35)
            hooks = m.decode(feat_i[0], feat_k[0], pos, gh, gw)
            pts, conf, d16, d32, dq = m.heads(hooks, gh, gw, H5, W5)
            if conc:
                main.wait_stream(s)
            r = U.apply_dynamic_mask_to_pointmaps(pts[0:2], conf[0:2], mask, d16, dq)
            r = list(r) if isinstance(r, (tuple, list)) else [r]
            torch.cuda.synchronize()
            outs.append([x.clone() for x in r if torch.is_tensor(x)] + [mask.clone(), Xm.clone()])
        for a, b in zip(*outs):
            assert torch.equal(a, b), ("fp8" if fp8 else "bf16")
    m.set_fp8(False)
