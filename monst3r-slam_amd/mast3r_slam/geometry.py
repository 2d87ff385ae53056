"""mast3r_slam.geometry (geometry.py:1-123): the host-side point / ray / projection helpers
of the tracker glue, restated in torch (the fused tracker kernels carry their own copies)."""
import torch


def skew_sym(x):
    z0 = torch.zeros_like(x[..., 0])
    a, b, c = x.unbind(-1)
    return torch.stack([z0, -c, b, c, z0, -a, -b, a, z0], -1).reshape(*x.shape[:-1], 3, 3)


def point_to_dist(X):
    return torch.linalg.norm(X, dim=-1, keepdim=True)


def point_to_ray_dist(X, jacobian=False):
    """(X / ‖X‖, ‖X‖) [..., 4] and, with jacobian, d(rd)/dX [..., 4, 3]."""
    d = point_to_dist(X)
    d_inv = 1.0 / d
    r = d_inv * X
    rd = torch.cat((r, d), -1)
    if not jacobian:
        return rd
    eye = torch.eye(3, device=X.device, dtype=X.dtype).expand(*X.shape[:-1], 3, 3)
    dr = d_inv[..., None] * (eye - (d_inv ** 2)[..., None] * (X[..., :, None] * X[..., None, :]))
    return rd, torch.cat((dr, r[..., None, :]), -2)


def get_pixel_coords(b, img_size, device, dtype):
    h, w = img_size
    v, u = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    return torch.stack((u, v), -1)[None].repeat(b, 1, 1, 1).to(device=device, dtype=dtype)


def backproject(p, z, K):
    x = (p[..., 0] - K[0, 2]) / K[0, 0]
    y = (p[..., 1] - K[1, 2]) / K[1, 1]
    ray = torch.stack((x, y, torch.ones_like(x)), -1).to(K.dtype)
    return z * ray


def constrain_points_to_ray(img_size, Xs, K):
    """Keep each pixel's depth, move the point onto the pixel's ray through K."""
    uv = get_pixel_coords(Xs.shape[0], img_size, Xs.device, Xs.dtype).view(*Xs.shape[:-1], 2)
    return backproject(uv, Xs[..., 2:3], K)


def act_Sim3(T, pC, jacobian=False):
    """T.act(pC) and, with jacobian, d(pW)/d(tangent) = [I, -[pW]x, pW] [..., 3, 7]."""
    pW = T.act(pC)
    if not jacobian:
        return pW
    eye = torch.eye(3, device=pW.device, dtype=pW.dtype).expand(*pW.shape[:-1], 3, 3)
    return pW, torch.cat((eye, -skew_sym(pW), pW[..., :, None]), -1)


def decompose_K(K):
    return K[..., 0, 0], K[..., 1, 1], K[..., 0, 2], K[..., 1, 2]


def project_calib(P, K, img_size, jacobian=False, border=0, z_eps=0.0):
    """(u, v, log z) of points P under K, validity (inside the border-shrunk image, z >
    z_eps) and, with jacobian, d(u, v, log z)/dP."""
    p = P @ K.T.to(P.dtype)
    uv = p[..., :2] / p[..., 2:3]
    u, v = uv[..., 0:1], uv[..., 1:2]
    x, y, z = P[..., 0:1], P[..., 1:2], P[..., 2:3]
    valid = ((u > border) & (u < img_size[1] - 1 - border) & (v > border) &
             (v < img_size[0] - 1 - border) & (z > z_eps))
    logz = torch.where(z > z_eps, torch.log(torch.where(z > z_eps, z, torch.ones_like(z))),
                       torch.zeros_like(z))
    pz = torch.cat((uv, logz), -1)
    if not jacobian:
        return pz, valid
    fx, fy, _, _ = decompose_K(K)
    zi = 1.0 / z[..., 0]
    J = torch.zeros(*P.shape[:-1], 3, 3, device=P.device, dtype=P.dtype)
    J[..., 0, 0] = fx * zi
    J[..., 1, 1] = fy * zi
    J[..., 0, 2] = -fx * x[..., 0] * zi * zi
    J[..., 1, 2] = -fy * y[..., 0] * zi * zi
    J[..., 2, 2] = zi
    return pz, J, valid
