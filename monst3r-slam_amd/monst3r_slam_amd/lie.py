"""lietorch-compatible Sim3 for the host-side SLAM glue (tracker2.py, global_opt2.py,
frame.py and main_monster_slam.py hold poses as `lietorch.Sim3`).  lietorch itself is a
git dependency of the reference (pyproject.toml:15) that is not installed offline; this is
the subset those callers use — `Sim3(data)`, `.data`, `Identity`, `inv`, `*`, `act`,
`retr`, `matrix`, indexing — on the same data layout [..., 8] = (t xyz, q xyzw, s) and
tangent order (tau, omega, sigma).  Formulas: lietorch's rxso3 / sim3 as restated in
gn_kernels.cu:178-413 (the same restatement the HIP kernels use, csrc/sim3.h).  These are
a few host-side ops per frame (7-dof poses, [N,3] point transforms), not the hot path: the
tracker / GN kernels do their Sim3 algebra on the device.

Reference callers may use it in place of lietorch:  `sys.modules["lietorch"] =
monst3r_slam_amd.lie` before importing them."""
from __future__ import annotations

import torch

_EPS = 1e-6


def _qmul(a, b):
    ax, ay, az, aw = a.unbind(-1)
    bx, by, bz, bw = b.unbind(-1)
    return torch.stack([aw * bx + ax * bw + ay * bz - az * by,
                        aw * by - ax * bz + ay * bw + az * bx,
                        aw * bz + ax * by - ay * bx + az * bw,
                        aw * bw - ax * bx - ay * by - az * bz], -1)


def _qact(q, X):
    """Rotate points X [..., 3] by unit quaternions q [..., 4] (broadcast)."""
    qv, qw = q[..., :3], q[..., 3:4]
    uv = 2.0 * torch.cross(qv.expand_as(X), X, dim=-1)
    return X + qw * uv + torch.cross(qv.expand_as(uv), uv, dim=-1)


def _exp(xi):
    """Sim3 exponential of tangent xi [..., 7] → data [..., 8] (csrc/sim3.h m3s_exp_sim3)."""
    xi = xi.to(torch.float64)
    tau, phi, sigma = xi[..., :3], xi[..., 3:6], xi[..., 6]
    th2 = (phi * phi).sum(-1)
    th = th2.sqrt()
    small = th2 < _EPS
    th_q = torch.where(small, torch.ones_like(th), th)     # so3 exp: Taylor below th^2 < EPS
    imag = torch.where(small, 0.5 - th2 / 48.0 + th2 * th2 / 3840.0, torch.sin(0.5 * th_q) / th_q)
    real = torch.where(small, 1.0 - th2 / 8.0 + th2 * th2 / 384.0, torch.cos(0.5 * th_q))
    q = torch.cat([imag[..., None] * phi, real[..., None]], -1)
    scale = torch.exp(sigma)
    sg_small = sigma.abs() < _EPS
    th_small = th.abs() < _EPS                              # sim3 V: Taylor below th < EPS
    th_s = torch.where(th_small, torch.ones_like(th), th)
    sg_s = torch.where(sg_small, torch.ones_like(sigma), sigma)
    C = torch.where(sg_small, torch.ones_like(sigma), (scale - 1.0) / sg_s)
    a = scale * torch.sin(th_s)
    b = scale * torch.cos(th_s)
    c = th2 + sigma * sigma
    A0 = torch.where(th_small, torch.full_like(th, 0.5), (1.0 - torch.cos(th_s)) / th_s ** 2)
    B0 = torch.where(th_small, torch.full_like(th, 1.0 / 6.0),
                     (th_s - torch.sin(th_s)) / (th_s ** 3))
    A1 = torch.where(th_small, ((sg_s - 1.0) * scale + 1.0) / sg_s ** 2,
                     (a * sg_s + (1.0 - b) * th_s) / (th_s * torch.where(c > 0, c, torch.ones_like(c))))
    B1 = torch.where(th_small,
                     (scale * 0.5 * sg_s ** 2 + scale - 1.0 - sg_s * scale) / sg_s ** 3,
                     (C - ((b - 1.0) * sg_s + a * th_s) / torch.where(c > 0, c, torch.ones_like(c)))
                     / th_s ** 2)
    A = torch.where(sg_small, A0, A1)
    B = torch.where(sg_small, B0, B1)
    c1 = torch.cross(phi, tau, dim=-1)
    c2 = torch.cross(phi, c1, dim=-1)
    t = C[..., None] * tau + A[..., None] * c1 + B[..., None] * c2
    return torch.cat([t, q, scale[..., None]], -1)


class Sim3:
    """lietorch.Sim3 subset; `data` [..., 8]."""

    def __init__(self, data):
        self.data = data.data if isinstance(data, Sim3) else data

    # -- construction --
    @classmethod
    def Identity(cls, *batch, device="cpu", dtype=torch.float32, requires_grad=False):
        d = torch.zeros((*batch, 8), device=device, dtype=dtype)
        d[..., 6] = 1.0
        d[..., 7] = 1.0
        return cls(d)

    @classmethod
    def exp(cls, xi):
        return cls(_exp(xi).to(xi.dtype))

    # -- structure --
    @property
    def shape(self):
        return self.data.shape[:-1]

    @property
    def device(self):
        return self.data.device

    def __getitem__(self, idx):
        return Sim3(self.data[idx])

    def __len__(self):
        return self.data.shape[0]

    def clone(self):
        return Sim3(self.data.clone())

    def to(self, *a, **k):
        return Sim3(self.data.to(*a, **k))

    def cpu(self):
        return Sim3(self.data.cpu())

    def __repr__(self):
        return f"Sim3({self.data})"

    # -- group operations --
    def _tqs(self):
        d = self.data
        return d[..., :3], d[..., 3:7], d[..., 7:8]

    def inv(self):
        t, q, s = self._tqs()
        qi = torch.cat([-q[..., :3], q[..., 3:]], -1)
        ti = -_qact(qi, t) / s
        return Sim3(torch.cat([ti, qi, 1.0 / s], -1))

    def __mul__(self, other):
        if not isinstance(other, Sim3):
            raise TypeError("Sim3 * Sim3 only (use act() for points)")
        t1, q1, s1 = self._tqs()
        t2, q2, s2 = other._tqs()
        return Sim3(torch.cat([t1 + s1 * _qact(q1, t2), _qmul(q1, q2), s1 * s2], -1))

    def act(self, X):
        """s R X + t on points [..., 3] (the pose broadcast over the leading dims of X)."""
        t, q, s = self._tqs()
        extra = X.dim() - t.dim()
        for _ in range(extra):
            t, q, s = t.unsqueeze(-2), q.unsqueeze(-2), s.unsqueeze(-2)
        return s * _qact(q, X) + t

    def retr(self, xi):
        """Left retraction Exp(xi) * X (lietorch retr)."""
        return Sim3(_exp(xi).to(self.data.dtype)) * self

    def matrix(self):
        t, q, s = self._tqs()
        x, y, z, w = q.unbind(-1)
        R = torch.stack([
            torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
            torch.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
            torch.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1)],
            -2) * s[..., None]
        M = torch.zeros((*t.shape[:-1], 4, 4), dtype=t.dtype, device=t.device)
        M[..., :3, :3] = R
        M[..., :3, 3] = t
        M[..., 3, 3] = 1.0
        return M


class SE3(Sim3):
    """The SE3 view lietorch_utils.as_SE3 produces (scale dropped to 1)."""
