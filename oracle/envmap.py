"""oracle/envmap.py — TEST INFRASTRUCTURE: the synthetic env map of the useEnvTex goldens and tests."""
import numpy as np


def synthetic_env(w=64, h=32):
    """The reference's env map (data/textures/veranda_1k.hdr) is not in the repository: a synthetic
    equirectangular RGBA8 sky instead (row 0 = up): blue zenith, bright horizon, brown ground, and a
    small sun disc."""
    v = (np.arange(h) + 0.5) / h
    u = (np.arange(w) + 0.5) / w
    V, U = np.meshgrid(v, u, indexing="ij")
    zen, hor, gnd = np.array([0.35, 0.55, 1.0]), np.array([0.95, 0.92, 0.85]), np.array([0.30, 0.24, 0.18])
    up = np.clip(1.0 - 2.0 * V, 0, 1)[..., None]
    dn = np.clip(2.0 * V - 1.0, 0, 1)[..., None]
    rgb = np.where(V[..., None] < 0.5, hor + (zen - hor) * up ** 0.6, hor + (gnd - hor) * dn ** 0.4)
    sun = ((U - 0.3) ** 2 + ((V - 0.22) * 0.5) ** 2) < 0.04 ** 2
    rgb[sun] = [1.0, 1.0, 0.92]
    out = np.empty((h, w, 4), np.uint8)
    out[..., :3] = np.round(rgb * 255.0).astype(np.uint8)
    out[..., 3] = 255
    return out
