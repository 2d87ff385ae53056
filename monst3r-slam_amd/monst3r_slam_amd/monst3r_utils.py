"""Model-level drop-in of mast3r_slam/monst3r_utils.py (and the frame helpers of
mast3r_slam/frame.py) on the MI355X pair model.

Same function names, argument order and return conventions as the reference, so the SLAM
glue (tracker2.py, global_opt2.py, main_monster_slam.py) reads the same:

  load_mast3r / load_monst3r              monst3r_utils.py:36-52
  monst3r_asymmetric_inference            :255-297   (frame i vs keyframe j)
  monst3r_match_asymmetric                :483-508   (+ matching.match)
  monst3r_symmetric_inference             :95-138
  monst3r_decode_symmetric_batch          :141-184   (true batching: chunked problem sets)
  monst3r_match_symmetric                 :214-252
  monst3r_inference_mono                  :187-211
  apply_dynamic_mask_to_pointmaps         :300-341   (HIP kernel m3s_apply_dynamic_mask)
  get_dynamic_mask                        :512-704   (caller's RAFT callable; mono decode,
                                                      ego flow, error mask on the GPU;
                                                      SAM2 refinement not provided)
  ego_flow / dynamic_mask_from_flow       :566-637   (DepthBasedWarping restated: unpinned)
  resize_img / create_frame / Frame       monst3r_utils.py:739-782, frame.py:14-141

Model handles: the reference keeps two nn.Modules; here both weight sets live in ONE
PairModel (both decoders and all heads run as one batched problem set), so
`load_monst3r` and `load_mast3r` return handles onto a shared model, built when the pair
is first used.  Weights: `path=None` → seeded random weights with the reference's
parameter names (no checkpoints offline); a path → the reference checkpoint format
({"model": state_dict}) read with torch.load(weights_only=True).
"""
from __future__ import annotations

import dataclasses
from typing import Optional

import numpy as np
import torch

from . import _lib
from . import matching
from . import model as Mdl
from . import weights as Wt
from .config import config

# ---------------------------------------------------------------------------------------
# model handles
# ---------------------------------------------------------------------------------------
_REGISTRY: dict = {}   # device str → {"monst3r": handle, "mast3r": handle}


class ModelHandle:
    """Stands for the reference's AsymmetricCroCo3DStereo (MonST3R) or AsymmetricMASt3R."""

    def __init__(self, kind, state_dict, arch, device):
        self.kind, self.sd, self.arch, self.device = kind, state_dict, arch, torch.device(device)
        self._pair_model = None

    def share_memory(self):        # main_monster_slam.py:206-207 (single process here)
        return self

    # ---- the reference model's methods (d3r/model.py:127-196), one model at a time ----
    def _encoder_model(self) -> Mdl.PairModel:
        """MonST3R's encoder is the pair model's; MASt3R's own encoder (used only when a
        caller encodes with the MASt3R handle) is packed on first use."""
        if self.kind == "monst3r":
            return self.pair_model()
        if getattr(self, "_enc_model", None) is None:
            # MASt3R's state dict in both slots: the encoder slot takes its encoder (its key
            # set is MonST3R's plus the local-feature MLP the second slot needs)
            self._enc_model = Mdl.PairModel(Mdl.PackedWeights(self.sd, self.arch, self.sd,
                                                              self.arch, self.device),
                                            self.device)
        return self._enc_model

    def _encode_image(self, image, true_shape):
        """d3r/model.py:127-139 → (feat [B,S,E] bf16, pos [B,S,2] int64, None)."""
        pm = self._encoder_model()
        feat, pos = pm.encode(image.to(self.device, torch.float32))
        return feat.clone(), pos.clone(), None

    def _decoder(self, f1, pos1, f2, pos2):
        """d3r/model.py:171-190 → (dec1, dec2): per view the 13 block outputs of this model's
        decoder; the MI355X decoder keeps only those the heads read — [0] (encoder tokens),
        [6], [9], [12] (dec_norm) — the other entries are None."""
        pm = self.pair_model()
        a = pm.a
        B, S = f1.shape[0], f1.shape[1]
        gh = int(pos1[0, :, 0].max()) + 1       # row count from the grid positions
        gw = S // gh
        hooks = pm.decode_multi(f1.to(Mdl.BF16).reshape(B, S, a.enc_dim),
                                f2.to(Mdl.BF16).reshape(B, S, a.enc_dim), gh, gw, models=2)
        m = 0 if self.kind == "monst3r" else 1
        idx = torch.arange(B, device=self.device) * 4 + m * 2   # z = (g*2 + model)*2 + side
        views = []
        for side in (0, 1):
            dec = [None] * (a.dec_depth + 1)
            for k in (0, 6, 9, 12):
                dec[k] = hooks[f"h{k}"][idx + side].clone()
            views.append(dec)
        return views[0], views[1]

    def _downstream_head(self, head_num, decout, img_shape):
        """d3r/model.py:192-196: head 1 / 2 of this model on one view's decoder outputs
        (bf16 heads; the reference runs them in f32, tolerances in tests/test_gpu_vit.py)."""
        pm = self.pair_model()
        H, W = _hw(img_shape)
        m = 0 if self.kind == "monst3r" else 1
        outs = []
        for b in range(decout[0].shape[0]):
            dec = {f"h{k}": decout[k][b:b + 1] for k in (0, 6, 9, 12)}
            outs.append(pm.single_head(dec, m, head_num - 1, H, W))
        return {k: torch.cat([o[k] for o in outs]) for k in outs[0]}

    def pair_model(self) -> Mdl.PairModel:
        reg = _REGISTRY.get(str(self.device), {})
        mon, mas = reg.get("monst3r"), reg.get("mast3r")
        if mon is None or mas is None:
            raise RuntimeError("load_monst3r() and load_mast3r() must both be called on this "
                               "device: the MI355X pair model batches both decoders")
        if mon._pair_model is None:
            pm = Mdl.PairModel(Mdl.PackedWeights(mon.sd, mon.arch, mas.sd, mas.arch,
                                                 self.device), self.device)
            mon._pair_model = mas._pair_model = pm
        return mon._pair_model


def _load_state_dict(path, arch, seed):
    if path is None:
        return Wt.make_state_dict(arch, seed)
    ck = torch.load(path, map_location="cpu", weights_only=True)
    sd = ck["model"] if isinstance(ck, dict) and "model" in ck else ck
    missing = set(Wt.param_shapes(arch)) - set(sd)
    if missing:
        raise RuntimeError(f"checkpoint {path} lacks {len(missing)} parameters, e.g. "
                           f"{sorted(missing)[:3]}")
    return {k: sd[k].float() for k in Wt.param_shapes(arch)}


def load_monst3r(path=None, device="cuda", arch=None):
    """monst3r_utils.py:46-52 (MonST3R_PO-TA-S-W_ViTLarge_BaseDecoder_512_dpt).
    `arch` (not in the reference) selects a reduced-width variant for tests."""
    a = arch or Wt.MONST3R
    h = ModelHandle("monst3r", _load_state_dict(path, a, 0), a, device)
    _REGISTRY.setdefault(str(h.device), {})["monst3r"] = h
    return h


def load_mast3r(path=None, device="cuda", arch=None):
    """monst3r_utils.py:36-43 (MASt3R_ViTLarge_BaseDecoder_512_catmlpdpt_metric)."""
    a = arch or Wt.MAST3R
    h = ModelHandle("mast3r", _load_state_dict(path, a, 1), a, device)
    _REGISTRY.setdefault(str(h.device), {})["mast3r"] = h
    return h


# ---------------------------------------------------------------------------------------
# frames (frame.py:14-141) and image preprocessing (monst3r_utils.py:739-782)
# ---------------------------------------------------------------------------------------
@dataclasses.dataclass
class Frame:
    """frame.py:14-50.  T_WC is the lietorch Sim3 data tensor [1,8] (t, q xyzw, s)."""
    frame_id: int
    img: torch.Tensor                 # [1,3,H,W] f32 in [-1,1]
    img_shape: torch.Tensor           # [1,2] int
    img_true_shape: torch.Tensor      # [1,2] int
    uimg: torch.Tensor                # [H,W,3] f32 in [0,1] (host)
    T_WC: Optional[torch.Tensor] = None
    X_canon: Optional[torch.Tensor] = None
    C: Optional[torch.Tensor] = None
    feat: Optional[torch.Tensor] = None   # [1,S,1024] bf16 (MonST3R encoder)
    pos: Optional[torch.Tensor] = None    # [1,S,2] int64
    N: int = 0
    N_updates: int = 0
    K: Optional[torch.Tensor] = None
    dynamic_mask: Optional[torch.Tensor] = None

    def update_pointmap(self, X, C):
        """frame.py:60-124, 'weighted_pointmap' (base.yaml:39) and the other modes that
        need no host statistics."""
        mode = config["tracking"]["filtering_mode"]
        if self.N == 0:
            self.X_canon, self.C, self.N, self.N_updates = X.clone(), C.clone(), 1, 1
            return
        if mode == "weighted_pointmap":
            self.X_canon = (self.C * self.X_canon + C * X) / (self.C + C)
            self.C = self.C + C
            self.N += 1
        elif mode == "recent":
            self.X_canon, self.C, self.N = X.clone(), C.clone(), 1
        elif mode == "first":
            if self.N_updates == 1:
                self.X_canon, self.C, self.N = X.clone(), C.clone(), 1
        elif mode == "indep_conf":
            m = C > self.C
            self.X_canon[m.repeat(1, 3)] = X[m.repeat(1, 3)]
            self.C[m] = C[m]
            self.N = 1
        else:
            raise NotImplementedError(f"filtering_mode {mode}")
        self.N_updates += 1

    def get_average_conf(self):
        return self.C / self.N if self.C is not None else None


def _resize_pil_image(img, long_edge_size):
    import PIL.Image
    S = max(img.size)
    interp = PIL.Image.LANCZOS if S > long_edge_size else PIL.Image.BICUBIC
    new_size = tuple(int(round(x * long_edge_size / S)) for x in img.size)
    return img.resize(new_size, interp)


def img_norm(pil_img):
    """dust3r ImgNorm = ToTensor + Normalize((0.5,)*3, (0.5,)*3) (d3r/utils/image.py:23)."""
    a = np.asarray(pil_img, dtype=np.float32) / 255.0
    return torch.from_numpy(((a - 0.5) / 0.5).transpose(2, 0, 1).copy())


def resize_img(img, size, square_ok=False, return_transformation=False):
    """monst3r_utils.py:749-782: long side → 512 (LANCZOS when shrinking, BICUBIC else)
    or short side → 224, then a centre crop to a multiple of 16 (4:3 for square inputs)."""
    import PIL.Image
    assert size == 224 or size == 512
    img = PIL.Image.fromarray(np.uint8(img * 255))
    W1, H1 = img.size
    if size == 224:
        img = _resize_pil_image(img, round(size * max(W1 / H1, H1 / W1)))
    else:
        img = _resize_pil_image(img, size)
    W, H = img.size
    cx, cy = W // 2, H // 2
    if size == 224:
        half = min(cx, cy)
        img = img.crop((cx - half, cy - half, cx + half, cy + half))
    else:
        halfw, halfh = ((2 * cx) // 16) * 8, ((2 * cy) // 16) * 8
        if not square_ok and W == H:
            halfh = 3 * halfw / 4
        img = img.crop((cx - halfw, cy - halfh, cx + halfw, cy + halfh))
    res = dict(img=img_norm(img)[None], true_shape=np.int32([img.size[::-1]]),
               unnormalized_img=np.asarray(img))
    if return_transformation:
        return res, (W1 / W, H1 / H, (W - img.size[0]) / 2, (H - img.size[1]) / 2)
    return res


def create_frame(i, img, T_WC, K=None, img_size=512, device="cuda:0"):
    """frame.py:130-141.  T_WC: Sim3 data [1,8] (or [8])."""
    r = resize_img(img, img_size)
    rgb = r["img"].to(device=device)
    img_shape = torch.tensor(r["true_shape"], device=device)
    img_true_shape = img_shape.clone()
    uimg = torch.from_numpy(r["unnormalized_img"].copy()) / 255.0
    ds = config["dataset"]["img_downsample"]
    if ds > 1:
        uimg = uimg[::ds, ::ds]
        img_shape = img_shape // ds
    T = torch.as_tensor(T_WC, dtype=torch.float32, device=device).reshape(1, 8)
    return Frame(i, rgb, img_shape, img_true_shape, uimg, T, K=K)


# ---------------------------------------------------------------------------------------
# inference
# ---------------------------------------------------------------------------------------
def _hw(frame_or_shape):
    s = frame_or_shape.img_true_shape if hasattr(frame_or_shape, "img_true_shape") \
        else frame_or_shape
    s = torch.as_tensor(s).reshape(-1)
    return int(s[0]), int(s[1])


def _ensure_feat(pm, frame):
    """Encode with MonST3R's encoder once and cache on the frame (monst3r_utils.py:262-269)."""
    if frame.feat is None:
        feat, pos = pm.encode(frame.img)
        frame.feat, frame.pos = feat.clone(), pos.clone()
    return frame.feat


def _downsample(*ts):
    """mast3r_downsample (monst3r_utils.py:82-91): [..., ::d, ::d(, :)]."""
    d = config["dataset"]["img_downsample"]
    if d <= 1:
        return ts
    out = []
    for t in ts:
        out.append(t[..., ::d, ::d, :].contiguous() if t.dim() >= 4 and t.shape[-1] in (3, 24)
                   else t[..., ::d, ::d].contiguous())
    return tuple(out)


@torch.inference_mode()
def monst3r_asymmetric_inference(mast3r, monst3r, frame_i, frame_j):
    """:255-297 → X, C (MonST3R heads) and D, Q (MASt3R heads), each [2,H,W(,c)]
    (index 0 = ii, 1 = ji); both decoders consume MonST3R encoder features."""
    pm = monst3r.pair_model()
    _ensure_feat(pm, frame_i)
    fj = _ensure_feat(pm, frame_j)
    H, W = _hw(frame_i)
    gh, gw = H // pm.a.patch, W // pm.a.patch
    hooks = pm.decode(frame_i.feat.reshape(-1, pm.a.enc_dim), fj.reshape(-1, pm.a.enc_dim),
                      None, gh, gw)
    pts, conf, _, desc, dconf = pm.heads(hooks, gh, gw, H, W)
    return _downsample(pts[0:2].clone(), conf[0:2].clone(), desc.clone(), dconf.clone())


def _rearrange_pair(X, C, D, Q):
    b = X.shape[0] // 2
    Xs = X.reshape(2, b, -1, 3)
    Cs = C.reshape(2, b, -1, 1)
    Ds = D.reshape(2, b, -1, D.shape[-1])
    Qs = Q.reshape(2, b, -1, 1)
    return Xs, Cs, Ds, Qs


def monst3r_match_asymmetric(mast3r, monst3r, frame_i, frame_j, idx_i2j_init=None):
    """:483-508 → (idx_i2j, valid_match_j, Xii, Cii, Qii, Xji, Cji, Qji)."""
    X, C, D, Q = monst3r_asymmetric_inference(mast3r, monst3r, frame_i, frame_j)
    b = X.shape[0] // 2
    idx_i2j, valid_match_j = matching.match(X[:b], X[b:], D[:b], D[b:],
                                            idx_1_to_2_init=idx_i2j_init)
    Xs, Cs, _, Qs = _rearrange_pair(X, C, D, Q)
    return idx_i2j, valid_match_j, Xs[0], Cs[0], Qs[0], Xs[1], Cs[1], Qs[1]


def monst3r_asymmetric_inference_with_dynamic_mask(mast3r, monst3r, frame_i, frame_j,
                                                   dynamic_mask_i=None, dynamic_mask_j=None):
    """:344-445 without the debug image dumps: the pair outputs with C / Q := 0 and D := 0
    where frame i's (view ii) or frame j's (view ji) dynamic mask is set."""
    X, C, D, Q = monst3r_asymmetric_inference(mast3r, monst3r, frame_i, frame_j)
    b = X.shape[0] // 2
    for mask, sl in ((dynamic_mask_i, slice(0, b)), (dynamic_mask_j, slice(b, 2 * b))):
        if mask is None:
            continue
        _, Cm, Dm, Qm = apply_dynamic_mask_to_pointmaps(X[sl], C[sl], mask, D[sl], Q[sl])
        C, D, Q = C.clone(), D.clone(), Q.clone()
        C[sl], D[sl], Q[sl] = Cm, Dm, Qm
    return X, C, D, Q


def monst3r_match_asymmetric_with_dynamic_mask(mast3r, monst3r, frame_i, frame_j,
                                               dynamic_mask_i=None, dynamic_mask_j=None,
                                               idx_i2j_init=None):
    """:448-480 → (idx_i2j, valid_match_j, Xii, Cii, Qii, Xji, Cji, Qji)."""
    X, C, D, Q = monst3r_asymmetric_inference_with_dynamic_mask(
        mast3r, monst3r, frame_i, frame_j, dynamic_mask_i, dynamic_mask_j)
    b = X.shape[0] // 2
    idx_i2j, valid_match_j = matching.match(X[:b], X[b:], D[:b], D[b:],
                                            idx_1_to_2_init=idx_i2j_init)
    Xs, Cs, _, Qs = _rearrange_pair(X, C, D, Q)
    return idx_i2j, valid_match_j, Xs[0], Cs[0], Qs[0], Xs[1], Cs[1], Qs[1]


@torch.inference_mode()
def monst3r_symmetric_inference(mast3r, monst3r, frame_i, frame_j):
    """:95-138 → X, C, D, Q [4,H,W(,c)] in the order (ii, ji, jj, ij)."""
    pm = monst3r.pair_model()
    fi, fj = _ensure_feat(pm, frame_i), _ensure_feat(pm, frame_j)
    H, W = _hw(frame_i)
    out = pm.symmetric(fi, fj, H, W)
    return _downsample(out["X"][:, 0], out["C"][:, 0], out["D"][:, 0], out["Q"][:, 0])


@torch.inference_mode()
def monst3r_decode_symmetric_batch(mast3r, monst3r, feat_i, pos_i, feat_j, pos_j, shape_i,
                                   shape_j, chunk=None):
    """:141-184 ("Assumes img shape the same") → X, C, D, Q [4,B,H,W(,c)].  The reference
    loops over b; here `chunk` pairs = 8·chunk decoder/head problems share every launch
    (None: PairModel.symmetric's near-equal chunks of at most `sym_chunk` pairs)."""
    pm = monst3r.pair_model()
    H, W = _hw(shape_i[0])
    out = pm.symmetric(feat_i.to(Mdl.BF16), feat_j.to(Mdl.BF16), H, W, chunk=chunk)
    return _downsample(out["X"], out["C"], out["D"], out["Q"])


def monst3r_match_symmetric(mast3r, monst3r, feat_i, pos_i, feat_j, pos_j, shape_i, shape_j):
    """:214-252 → (idx_i2j, idx_j2i, valid_match_j, valid_match_i, Qii, Qjj, Qji, Qij).
    (global_opt2.py:54 omits `mast3r` — SURVEY §0.6a; here it is required, as in
    global_opt.py:49-50.)"""
    X, C, D, Q = monst3r_decode_symmetric_batch(mast3r, monst3r, feat_i, pos_i, feat_j,
                                                pos_j, shape_i, shape_j)
    b = X.shape[1]
    X11 = torch.cat((X[0], X[2]), 0)
    X21 = torch.cat((X[1], X[3]), 0)
    D11 = torch.cat((D[0], D[2]), 0)
    D21 = torch.cat((D[1], D[3]), 0)
    idx_1_to_2, valid_match_2 = matching.match(X11, X21, D11, D21)
    idx_i2j, idx_j2i = idx_1_to_2[:b], idx_1_to_2[b:]
    valid_match_j, valid_match_i = valid_match_2[:b], valid_match_2[b:]
    return (idx_i2j, idx_j2i, valid_match_j, valid_match_i, Q[0].reshape(b, -1, 1),
            Q[2].reshape(b, -1, 1), Q[1].reshape(b, -1, 1), Q[3].reshape(b, -1, 1))


@torch.inference_mode()
def monst3r_inference_mono(monst3r, frame):
    """:187-211 → (Xii [1,N,3], Cii [1,N,1])."""
    pm = monst3r.pair_model()
    f = _ensure_feat(pm, frame)
    H, W = _hw(frame)
    X, C = pm.mono(f, H, W)
    X, C = _downsample(X.clone(), C.clone())
    return X[0:1].reshape(1, -1, 3), C[0:1].reshape(1, -1, 1)


# ---------------------------------------------------------------------------------------
# dynamic mask (monst3r_utils.py:300-341, 512-704)
# ---------------------------------------------------------------------------------------
def _quat_rot(q):
    x, y, z, w = q.unbind(-1)
    return torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
        torch.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
        torch.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)], -2)


def sim3_relative_matrix(T_WC_i, T_WC_j):
    """lietorch (T_WC_j.inv() * T_WC_i).matrix()[:3] for data tensors [..., 8] (t, q xyzw,
    s): returns (sR [3,3], t [3]) of T_ji (:566-578), device tensors, no host sync."""
    Ti, Tj = T_WC_i.reshape(8).float(), T_WC_j.reshape(8).float()
    Ri, Rj = _quat_rot(Ti[3:7]), _quat_rot(Tj[3:7])
    si, sj = Ti[7], Tj[7]
    # T_j^-1 T_i: x → (Rj^T (si Ri x + ti - tj)) / sj
    sR = (si / sj) * (Rj.t() @ Ri)
    t = (Rj.t() @ (Ti[:3] - Tj[:3])) / sj
    return sR, t


def _inv3(K):
    """3x3 inverse by the adjugate (elementwise torch ops: no solver call, graph-capturable)."""
    a, b, c, d, e, f, g, h, i = K.reshape(9).unbind()
    co = torch.stack([e * i - f * h, c * h - b * i, b * f - c * e,
                      f * g - d * i, a * i - c * g, c * d - a * f,
                      d * h - e * g, b * g - a * h, a * e - b * d]).reshape(3, 3)
    return co / (a * co[0, 0] + b * co[1, 0] + c * co[2, 0])


def ego_flow(pts_i, R_ji, t_ji, K_j, K_i):
    """Ego-motion flow of frame i's pixels into frame j (the DepthBasedWarping call of
    :597-604) from the mono pointmap pts_i [..,H,W,3] (depth = z): ego f32 [3,H,W]
    (flow x, flow y, valid).  HIP kernel m3s_ego_flow; the warp is restated (its source is
    not in the reference checkout: parity unpinned)."""
    H, W = pts_i.shape[-3:-1]
    p = pts_i.reshape(H, W, 3).float().contiguous()
    _lib.require_cuda(p, names=("pts_i",))
    prm = torch.cat([R_ji.reshape(9).float(), t_ji.reshape(3).float(),
                     K_j.reshape(9).float(), _inv3(K_i.reshape(3, 3).float()).reshape(9)
                     ]).to(p.device).contiguous()
    ego = torch.empty((3, H, W), dtype=torch.float32, device=p.device)
    _lib.check(_lib.load().m3s_ego_flow(_lib.ptr(p), _lib.ptr(prm), H, W, _lib.ptr(ego),
                                        _lib.stream(p.device)), "ego_flow")
    return ego


@torch.inference_mode()
def get_dynamic_mask(monst3r, raft_model, frame_i, frame_j, threshold=0.35,
                     refine_with_sam2=True, sam2_predictor=None):
    """:512-704.  raft_model: the caller's RAFT (called as the reference does,
    raft_model(img_i_255, img_j_255, iters=20, test_mode=True)[1] → flow [1,2,H,W]); the
    depth comes from the MonST3R-only mono decode of frame i (res_i pts3d z, :580-587).
    Returns bool [H,W]; an all-False mask when K is missing or the flow call fails, like
    the reference.  SAM2 refinement needs the absent SAM2 predictor: requesting it with
    a predictor raises NotImplementedError (the unrefined mask is what the reference
    returns when no predictor is given)."""
    H, W = _hw(frame_i)
    dev = frame_i.img.device
    empty = torch.zeros((H, W), dtype=torch.bool, device=dev)
    if getattr(frame_i, "K", None) is None or getattr(frame_j, "K", None) is None:
        return empty
    try:
        img_i = frame_i.img if frame_i.img.dim() == 4 else frame_i.img[None]
        img_j = frame_j.img if frame_j.img.dim() == 4 else frame_j.img[None]
        flow = raft_model((img_i * 0.5 + 0.5) * 255.0, (img_j * 0.5 + 0.5) * 255.0, iters=20,
                          test_mode=True)[1].reshape(2, H, W)
    except Exception as e:  # the reference prints and returns the empty mask
        print(f"Error computing optical flow: {e}")
        return empty
    sR, t = sim3_relative_matrix(frame_i.T_WC, frame_j.T_WC)
    pm = monst3r.pair_model()
    f = _ensure_feat(pm, frame_i)
    X, _ = pm.mono(f, H, W)
    ego = ego_flow(X[0], sR, t, frame_j.K, frame_i.K)
    mask = dynamic_mask_from_flow(flow, ego, threshold)
    if refine_with_sam2 and sam2_predictor is not None:
        raise NotImplementedError("SAM2 refinement (:640-700) needs the SAM2 predictor, "
                                  "which is not part of this package")
    return mask


def dynamic_mask_from_flow(flow_ij, ego_flow_ij, threshold=0.35):
    """The mask arithmetic of get_dynamic_mask (:625-637): err = |flow - ego_flow[:2]|,
    min-max normalised, > threshold.  flow f32 [2,H,W], ego [>=2,H,W] → bool [H,W].
    (RAFT optical flow, DepthBasedWarping ego-flow and SAM2 refinement are absent from the
    reference checkout: their parity is unpinned; the inputs here come from the caller.)"""
    _lib.require_cuda(flow_ij, ego_flow_ij, names=("flow_ij", "ego_flow_ij"))
    f = flow_ij.float().contiguous()
    e = ego_flow_ij[:2].float().contiguous()
    H, W = f.shape[-2:]
    mask = torch.empty((H, W), dtype=torch.uint8, device=f.device)
    ws = torch.empty((H * W + 64,), dtype=torch.float32, device=f.device)
    _lib.check(_lib.load().m3s_flow_error_mask(_lib.ptr(f), _lib.ptr(e), H * W,
                                               float(threshold), _lib.ptr(mask), _lib.ptr(ws),
                                               _lib.stream(f.device)), "flow_error_mask")
    return mask.bool()


def apply_dynamic_mask_to_pointmaps(X, C, dynamic_mask, D=None, Q=None,
                                    mask_confidence_value=0.0, zero_descriptors=True):
    """:300-341: C (and Q) := value and D := 0 where the mask is set; X unchanged.
    X [b,h,w,3], C [b,h,w], D [b,h,w,F], Q [b,h,w], mask bool [h,w].  Returns new tensors
    (the reference clones); the fill is one fused HIP pass."""
    if dynamic_mask is None:
        return X, C, D, Q
    _lib.require_cuda(C, dynamic_mask, names=("C", "dynamic_mask"))
    Cm = C.float().contiguous().clone()
    Qm = None if Q is None else Q.float().contiguous().clone()
    Dm = None if D is None else D.contiguous().clone()
    b = Cm.shape[0]
    hw = Cm[0].numel()
    m = dynamic_mask.reshape(-1).to(torch.uint8).contiguous()
    fdim = 0 if Dm is None else Dm.shape[-1]
    is16 = int(Dm is not None and Dm.dtype == torch.float16)
    _lib.check(_lib.load().m3s_apply_dynamic_mask(
        _lib.ptr(m), _lib.ptr(Cm), _lib.ptr(Qm), _lib.ptr(Dm), is16, b, hw, fdim,
        float(mask_confidence_value), int(bool(zero_descriptors)), _lib.stream(C.device)),
        "apply_dynamic_mask")
    return X, Cm, Dm, Qm
