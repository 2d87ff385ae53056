"""Where does the fp8 (C5) path's error come from?  (tools only, round 5)

Fake-quantised fp32 restatement of the MonST3R mono decode at 512x512 (the C5 dyn-mask
decode, oracle/vit_ref.py's encode + inference_mono) with the fp8 path's roundings placed
where the HIP path places them (monst3r_slam_amd/model.py ENC_FP8 / DEC_FP8):
  weights   per-output-row e4m3, scale = amax / 448           (model.quant_e4m3)
  ln        e4m3 of each LayerNorm output feeding an fp8 GEMM  (unit scale)
  attn      e4m3 of the attention output feeding proj / cproj (unit scale)
  gelu      e4m3 of the GELU hidden feeding fc2                (unit scale)
Every site can be switched on alone, so the table shows each site's share of the pointmap
error (X median relative error vs the unquantised restatement, as the GPU test measures
it) and the share of each site's values that fall below e4m3's smallest normal (2^-6).
A site can also be given a static power-of-two pre-scale ('ln*16' etc.): values are
multiplied before rounding and divided after (the dequant the GEMM's column scale would
absorb).
Usage: python tools/fp8_error_budget.py [site-set ...]   e.g.  weights ln attn gelu all
       (default: each site alone, then all)   env DEV=cuda to run on a GPU, SIZE=512"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd import weights as Wt  # noqa: E402
from oracle import vit_ref as V  # noqa: E402

DEV = os.environ.get("DEV", "cpu")
SIZE = int(os.environ.get("SIZE", "512"))
torch.set_num_threads(os.cpu_count() or 8)
torch.backends.cuda.matmul.allow_tf32 = False

E4M3_MIN_NORMAL = 2.0 ** -6
CAL = {}                                   # GEMM name -> calibrated input mean
NCAL = int(os.environ.get("NCAL", "2"))    # calibration frames (seeds 100, 101, ...)


def e4m3(x):
    return x.clamp(-448.0, 448.0).to(torch.float8_e4m3fn).float()


class Q:
    """Active fake-quant sites and their statistics."""

    def __init__(self, sites):
        self.scale = {}
        self.sites = set()
        for s in sites:
            name, _, sc = s.partition("*")
            self.sites.add(name)
            if sc:
                self.scale[name] = float(sc)
        self.stats = {}

    def act(self, x, site, name=None):
        if site not in self.sites:
            return x
        if ("shift" in self.sites or ("shiftng" in self.sites and site != "gelu")) and name in CAL:
            # quantise x - mu (mu folded into params)
            mu = CAL[name]
            return e4m3(x - mu) + mu
        ax = x.abs()
        st = self.stats.setdefault(site, [0, 0, 0.0])
        st[0] += ax.numel()
        st[1] += int((ax < E4M3_MIN_NORMAL).sum())
        st[2] = max(st[2], float(ax.max()))
        s = self.scale.get(site, 1.0)
        return e4m3(x * s) / s

    def lin(self, x, sd, name, site, ex=None):
        """ex: the data-free expectation of the input per channel (bias correction 'bc')."""
        if "record" in self.sites:          # calibration pass (unquantised): input means
            m = x.reshape(-1, x.shape[-1]).mean(0)
            CAL[name] = CAL.get(name, 0) + m / NCAL
        w = sd[name + ".weight"]
        b = sd.get(name + ".bias")
        if "weights" in self.sites:
            sc = (w.abs().amax(-1) / 448.0).clamp_min(1e-12)
            wq = e4m3(w / sc[:, None]) * sc[:, None]
            if "bc_emp" in self.sites:      # upper bound: the input's own mean over tokens
                ex = x.reshape(-1, x.shape[-1]).mean(0)
            elif "bc_cal" in self.sites:    # calibrated: the mean recorded on other frames
                ex = CAL[name]
            elif "bc" not in self.sites:
                ex = None
            if ex is not None:               # E[(Wq - W) x] removed through the bias
                b = b - (wq - w) @ ex
            w = wq
        return F.linear(self.act(x, site, name), w, b)


# Data-free input expectations (the DFQ bias-correction estimates: LayerNorm output
# ~ beta per channel; attention output ~ E[v] since softmax rows sum to 1; GELU of a
# Gaussian pre-activation N(W1 beta + b1, sum_k W1^2 gamma^2) in closed form)
def _gelu_gauss_mean(mu, var):
    s = (var + 1.0).sqrt()
    z = mu / s
    pdf = torch.exp(-0.5 * z * z) / (2 * torch.pi) ** 0.5
    cdf = 0.5 * (1 + torch.erf(z / 2 ** 0.5))
    return mu * cdf + var / s * pdf


def _ex_ln(sd, ln):
    return sd[ln + ".bias"]


def _ex_attn(sd, wname, bname, ln, rows):
    w = sd[wname][rows]
    b = sd[bname][rows]
    return w @ sd[ln + ".bias"] + b


def _ex_gelu(sd, fc1, ln):
    w, b = sd[fc1 + ".weight"], sd[fc1 + ".bias"]
    mu = w @ sd[ln + ".bias"] + b
    var = (w * w) @ (sd[ln + ".weight"] ** 2)
    return _gelu_gauss_mean(mu, var)


def self_attention(q8, x, pos, sd, name, heads, base, ln):
    B, N, C = x.shape
    qkv = q8.lin(x, sd, name + ".qkv", "ln", _ex_ln(sd, ln)).reshape(B, N, 3, heads, C // heads)
    qkv = qkv.transpose(1, 3)
    q, k, v = [qkv[:, :, i] for i in range(3)]
    o = V._attn(q, k, v, pos, pos, base).transpose(1, 2).reshape(B, N, C)
    ex = _ex_attn(sd, name + ".qkv.weight", name + ".qkv.bias", ln, slice(2 * C, 3 * C))
    return q8.lin(o, sd, name + ".proj", "attn", ex)


def cross_attention(q8, x, y, xpos, ypos, sd, name, heads, base, ln, lny):
    B, Nq, C = x.shape
    Nk = y.shape[1]
    q = q8.lin(x, sd, name + ".projq", "ln", _ex_ln(sd, ln)).reshape(B, Nq, heads, C // heads)
    k = q8.lin(y, sd, name + ".projk", "ln", _ex_ln(sd, lny)).reshape(B, Nk, heads, C // heads)
    v = q8.lin(y, sd, name + ".projv", "ln", _ex_ln(sd, lny)).reshape(B, Nk, heads, C // heads)
    q, k, v = (t.permute(0, 2, 1, 3) for t in (q, k, v))
    o = V._attn(q, k, v, xpos, ypos, base).transpose(1, 2).reshape(B, Nq, C)
    ex = _ex_attn(sd, name + ".projv.weight", name + ".projv.bias", lny, slice(None))
    return q8.lin(o, sd, name + ".proj", "attn", ex)


def mlp(q8, x, sd, name, ln):
    h = F.gelu(q8.lin(x, sd, name + ".fc1", "ln", _ex_ln(sd, ln)))
    return q8.lin(h, sd, name + ".fc2", "gelu", _ex_gelu(sd, name + ".fc1", ln))


def encode(q8, sd, arch, img):
    B, _, H, W = img.shape
    x = F.conv2d(img, sd["patch_embed.proj.weight"], sd["patch_embed.proj.bias"], stride=arch.patch)
    gh, gw = x.shape[-2:]
    x = x.flatten(2).transpose(1, 2)
    pos = V.positions(B, gh, gw, img.device)
    for i in range(arch.enc_depth):
        p = f"enc_blocks.{i}."
        x = x + self_attention(q8, V._ln(x, sd, p + "norm1"), pos, sd, p + "attn", arch.enc_heads,
                               arch.rope_base, p + "norm1")
        x = x + mlp(q8, V._ln(x, sd, p + "norm2"), sd, p + "mlp", p + "norm2")
    return V._ln(x, sd, "enc_norm"), pos


def decoder_block(q8, x, y, xpos, ypos, sd, p, heads, base):
    x = x + self_attention(q8, V._ln(x, sd, p + "norm1"), xpos, sd, p + "attn", heads, base,
                           p + "norm1")
    y_ = V._ln(y, sd, p + "norm_y")
    x = x + cross_attention(q8, V._ln(x, sd, p + "norm2"), y_, xpos, ypos, sd, p + "cross_attn",
                            heads, base, p + "norm2", p + "norm_y")
    return x + mlp(q8, V._ln(x, sd, p + "norm3"), sd, p + "mlp", p + "norm3")


def mono(q8, sd, arch, img, H, W):
    feat, pos = encode(q8, sd, arch, img)
    return (feat,) + decode_mono(q8, sd, arch, feat, pos, H, W)


def decode_mono(q8, sd, arch, feat, pos, H, W):
    f1 = V._lin(feat, sd, "decoder_embed")
    out = [(f1, f1)]
    for i in range(arch.dec_depth):
        a, b = out[-1]
        out.append((decoder_block(q8, a, b, pos, pos, sd, f"dec_blocks.{i}.", arch.dec_heads,
                                  arch.rope_base),
                    decoder_block(q8, b, a, pos, pos, sd, f"dec_blocks2.{i}.", arch.dec_heads,
                                  arch.rope_base)))
    out = [(feat, feat)] + out[1:]
    out[-1] = tuple(V._ln(t, sd, "dec_norm") for t in out[-1])
    r = V.head(sd, arch, 1, [o[0] for o in out], H, W)
    return r["pts3d"].reshape(-1, 3), r["conf"].reshape(-1)


@torch.no_grad()
def main():
    am = Wt.MONST3R
    sd = {k: v.to(DEV) for k, v in Wt.make_state_dict(am, 0).items()}
    gen = torch.Generator(device=DEV).manual_seed(9)
    img = torch.rand(1, 3, SIZE, SIZE, device=DEV, generator=gen) * 2 - 1
    f0, X0, C0 = mono(Q([]), sd, am, img, SIZE, SIZE)
    print(f"mono {SIZE}x{SIZE}: median |X| {float(X0.norm(dim=-1).median()):.4f}, "
          f"median C {float(C0.median()):.4f}", flush=True)
    if any("bc_cal" in a or "shift" in a for a in sys.argv[1:]):  # shift, shiftng
        for c in range(NCAL):
            g2 = torch.Generator(device=DEV).manual_seed(100 + c)
            im = torch.rand(1, 3, SIZE, SIZE, device=DEV, generator=g2) * 2 - 1
            mono(Q(["record"]), sd, am, im, SIZE, SIZE)
    runs = [a.split("+") for a in sys.argv[1:]] or \
        [["weights"], ["ln"], ["attn"], ["gelu"], ["weights", "ln", "attn", "gelu"]]
    for sites in runs:
        if "all" in sites:
            sites = [x for x in sites if x != "all"] + ["weights", "ln", "attn", "gelu"]
        q8 = Q(sites)
        f, X, C = mono(q8, sd, am, img, SIZE, SIZE)
        rel_X = (X - X0).norm(dim=-1) / X0.norm(dim=-1).clamp_min(1e-6)
        rel_C = (C - C0).abs() / C0.abs()
        cos_f = F.cosine_similarity(f.reshape(-1, f.shape[-1]), f0.reshape(-1, f0.shape[-1]), -1)
        sub = " ".join(f"{k}: {v[1] / max(v[0], 1):.3f} sub, amax {v[2]:.1f}"
                       for k, v in sorted(q8.stats.items()))
        print(f"{'+'.join(sites):32s} X_med {float(rel_X.median()):.4f}  C_med "
              f"{float(rel_C.median()):.5f}  feat_cos_med {float(cos_f.median()):.5f}  [{sub}]",
              flush=True)


if __name__ == "__main__":
    main()
