"""The claim kernel's division-free decision (K5a, xrs_rectify.hip
tri_forms2 / walk_pair) restated in numpy float32 and checked against the
reference's float64 triangle test (rectify.py:544-573) on random and
adversarial quads: a pixel the float32 forms call surely-A / surely-B /
surely-miss must be exactly that for the reference, and every pixel of the
reference's window outside the trimmed window must be a miss of both
triangles.  This pins the error bound M (and the determinant threshold) the
kernel relies on; the kernel itself is checked against the oracle by
test_rectify_gpu.py.

The restatement follows the kernel's operation order (no contraction except
its explicit FMAs; the reciprocal is nudged by up to 1 ulp as v_rcp_f32 may
be)."""

from __future__ import annotations

import numpy as np
import pytest

F32 = np.float32
UV_DELTA = 1e-3          # constants.py UV_DELTA (rectify.py:483-484)
K_MAX_FORM_MARGIN = 1e-3  # xrs_rectify.hip kMaxFormMargin
K_PAD_EPS32 = 2.0 ** -20  # xrs_rectify.hip kPadEps32
K_LANE_WINDOW = 16


def f32(x):
    return np.asarray(x, dtype=np.float64).astype(F32)


def fma(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(F32)


# -- the reference's float64 test (rectify.py:742-763, 556-573) ----------------
def _fdet(x0, y0, x1, y1, x2, y2):
    return (x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)


def _fu(px, py, x0, y0, x2, y2):
    return (x0 - px) * (y0 - y2) - (y0 - py) * (x0 - x2)


def _fv(px, py, x0, y0, x1, y1):
    return (y0 - py) * (x0 - x1) - (x0 - px) * (y0 - y1)


def ref_choice(P, dx, dy):
    """1 = A hits, 2 = A misses and B hits, 0 = neither; P: (4, 2, N) corner
    coordinates p0..p3, dx, dy: (N, K) pixel centres."""
    umin, uvmax = -UV_DELTA, 1.0 + 2 * UV_DELTA
    (x0, y0), (x1, y1), (x2, y2), (x3, y3) = [(P[k, 0][:, None], P[k, 1][:, None])
                                              for k in range(4)]
    with np.errstate(all="ignore"):
        da = _fdet(x0, y0, x1, y1, x2, y2)
        db = _fdet(x3, y3, x2, y2, x1, y1)
        ua = _fu(dx, dy, x0, y0, x2, y2) / da
        va = _fv(dx, dy, x0, y0, x1, y1) / da
        ub = _fu(dx, dy, x3, y3, x1, y1) / db
        vb = _fv(dx, dy, x3, y3, x2, y2) / db
        hit_a = (da != 0) & (da == da) & (ua >= umin) & (va >= umin) & (ua + va <= uvmax)
        hit_b = (db != 0) & (db == db) & (ub >= umin) & (vb >= umin) & (ub + vb <= uvmax)
    return np.where(hit_a, 1, np.where(hit_b, 2, 0))


# -- the kernel's float32 forms ---------------------------------------------------
K_EPS32, K_EPS64 = 2.0 ** -23, 2.0 ** -52


def forms2(ex, ey, e1, e2, e3, e4, sx, sy, XY2, G0, rng):
    """tri_forms2 for one triangle (arrays over quads; ex .. e4 the float64
    corner differences in coordinate units): (u0, ui, uj, v0, vi, vj, w0, wi,
    wj, thr) and the status (1 forms set up, 0 no triangle, -1 exact test)."""
    umin, uvmax = f32(-UV_DELTA), f32(1.0 + 2 * UV_DELTA)
    det = e3 * e1 - e2 * e4
    with np.errstate(invalid="ignore"):
        tri = ~((det != det) | (det == 0.0))
    fex, fey, f1, f2, f3, f4 = (f32(v) for v in (ex, ey, e1, e2, e3, e4))
    with np.errstate(all="ignore"):
        fr = f32(1.0 / f32(det).astype(np.float64))
    nudge = rng.integers(-1, 2, size=fr.shape)   # v_rcp_f32: within 1 ulp
    fr = np.where(nudge > 0, np.nextafter(fr, F32(np.inf)),
                  np.where(nudge < 0, np.nextafter(fr, F32(-np.inf)), fr)).astype(F32)
    fS = f32((np.abs(e1) + np.abs(e2)) + (np.abs(e3) + np.abs(e4)))
    fxy = f32(np.abs(ex) + np.abs(ey))
    with np.errstate(all="ignore"):
        u0 = (fex * f1 - fey * f2) * fr
        v0 = (fey * f3 - fex * f4) * fr
        sxr, syr = sx * fr, sy * fr
        ui, uj, vi, vj = -(sxr * f1), syr * f2, sxr * f4, -(syr * f3)
        Sr = fS * np.abs(fr)
        P, G = fxy * Sr, G0 * Sr
        T = P + G
        E = F32(16) * P + (F32(14) * G + F32(24))
        R = (XY2 + fxy) * Sr
        M = (F32(K_EPS32) * E + F32(K_EPS64) * (F32(10) * R + F32(8) * T)) * F32(2.02)
        st = np.where(~tri, 0, np.where(M <= F32(K_MAX_FORM_MARGIN), 1, -1))
        forms = [(u0 - umin) - M, ui, uj, (v0 - umin) - M, vi, vj, (uvmax - (u0 + v0)) - M,
                 -(ui + vi), -(uj + vj), F32(-2) * M]
    forms[0] = np.where(tri, forms[0], F32(-np.inf)).astype(F32)   # never hits
    for k in (1, 2, 3, 4, 5, 6, 7, 8, 9):
        forms[k] = np.where(tri, forms[k], F32(0)).astype(F32)
    return tuple(forms), st


def walk_codes(FA, FB, nw, af, bf):
    """walk_pair's code per pixel (af, bf: (N, K) window column / row)."""
    def mins(F):
        u0, ui, uj, v0, vi, vj, w0, wi, wj, _ = [f[:, None] for f in F]
        u = fma(bf, uj, fma(af, ui, u0))
        v = fma(bf, vj, fma(af, vi, v0))
        w = fma(bf, wj, fma(af, wi, w0))
        return np.minimum(u, np.minimum(v, w))
    ha, hb = mins(FA), mins(FB)
    ta, tb = FA[9][:, None], FB[9][:, None]
    a_in, a_near = ha >= 0, ha >= ta
    return np.where(a_in, 1, np.where(~a_near & (hb >= 0), 2,
                                      np.where(a_near | (hb >= tb), 3, 0)))


GEOMETRIES = [   # (x_off, x_scale, y_off, y_scale): tile origins and pixel sizes
    (10.123456789, 0.0025, 60.0, -0.0025),
    (-179.875, 1.0 / 3600.0, 89.5, -1.0 / 3600.0),
    (500000.0, 300.0, 7.0e6, -300.0),
    (-2.0e7, 1.0 / 3.0, 1.0e7, 0.1),
]


def _quads(rng, n, adversarial):
    """Corner positions in target pixel units (tile-local), (4, 2, n)."""
    c = rng.uniform(40.0, 2000.0, size=(2, n))
    if not adversarial:
        s = np.exp(rng.uniform(np.log(0.03), np.log(2.6), size=n))
        th = rng.uniform(0, 2 * np.pi, size=n)
        sk = rng.uniform(0.4, 1.6, size=n)
        d1 = s * np.array([np.cos(th), np.sin(th)])
        d2 = s * sk * np.array([-np.sin(th + 0.3 * (sk - 1)), np.cos(th + 0.3 * (sk - 1))])
        p0 = c
        p1, p2 = p0 + d1, p0 + d2
        p3 = p1 + d2 + s * rng.normal(0, 0.15, size=(2, n))
        return np.stack([p0, p1, p2, p3])
    # axis-aligned quads whose edges pass a pixel centre at the reference's
    # decision boundaries (u = umin, v = umin, u + v = uvmax) plus a tiny delta
    L = rng.choice([0.5, 1.0, 1.5, 2.0], size=n)
    H = rng.choice([0.5, 1.0, 2.0], size=n)
    delta = rng.choice([0.0, 1e-13, -1e-13, 1e-10, -1e-10, 1e-7, -1e-7, 1e-5, -1e-5], size=n)
    cx, cy = np.floor(c) + 0.5
    kind = rng.integers(0, 3, size=n)
    # u = (x - p0x) / L, v = (y - p0y) / H for triangle A with p1 = p0 + (L, 0),
    # p2 = p0 + (0, H): put the centre (cx, cy) at the boundary of the kind
    uc = np.where(kind == 0, -UV_DELTA + delta, rng.uniform(0.0, 0.5, size=n))
    vc = np.where(kind == 1, -UV_DELTA + delta,
                  np.where(kind == 2, 1.0 + 2 * UV_DELTA - uc - delta, rng.uniform(0.0, 0.5, size=n)))
    p0 = np.array([cx - uc * L, cy - vc * H])
    p1 = p0 + np.array([L, np.zeros(n)])
    p2 = p0 + np.array([np.zeros(n), H])
    p3 = p0 + np.array([L, H])
    return np.stack([p0, p1, p2, p3])


@pytest.mark.parametrize("geo", range(len(GEOMETRIES)))
@pytest.mark.parametrize("adversarial", [False, True])
def test_float32_forms_decide_like_the_reference(geo, adversarial):
    rng = np.random.default_rng(1000 + 10 * geo + adversarial)
    x_off, x_scale, y_off, y_scale = GEOMETRIES[geo]
    tw = th = 2048
    n = 20000
    Qt = _quads(rng, n, adversarial)
    # the source coordinates (the data): float64 coordinates of those points
    P = np.empty_like(Qt)
    P[:, 0] = x_off + Qt[:, 0] * x_scale
    P[:, 1] = y_off + Qt[:, 1] * y_scale
    inv_x, inv_y = 1.0 / x_scale, 1.0 / y_scale
    # the kernel's tile-local pixel units, float32 (window extremes, pair_q)
    qx = f32((P[:, 0] - x_off) * inv_x)
    qy = f32((P[:, 1] - y_off) * inv_y)
    qx0, qx1 = qx.min(0), qx.max(0)
    qy0, qy1 = qy.min(0), qy.max(0)
    sq = (np.abs(qx0) + np.abs(qx1)) + (np.abs(qy0) + np.abs(qy1))
    d = f32(UV_DELTA + K_MAX_FORM_MARGIN)
    pad = F32(8) * d * ((qx1 - qx0) + (qy1 - qy0)) + F32(1e-6 + K_PAD_EPS32) * (F32(1) + sq)
    lo, hi = F32(0.5) + pad, F32(0.5) - pad
    ci, fi = np.ceil(qx0 - lo), np.floor(qx1 - hi)      # trimmed window T
    cj, fj = np.ceil(qy0 - lo), np.floor(qy1 - hi)
    ci, fi, cj, fj = (v.astype(np.float64) for v in (ci, fi, cj, fj))   # integers
    nw, nh = fi - ci + 1, fj - cj + 1
    cnt = np.where((nw > 0) & (nh > 0), nw * nh, 0)
    walk = (pad < 0.25) & (cnt > 0) & (cnt <= K_LANE_WINDOW)
    sxf, syf = F32(x_scale), F32(y_scale)
    XY2 = F32(2) * max(np.abs(F32(x_off)) + F32(tw + 1) * np.abs(sxf),
                       np.abs(F32(y_off)) + F32(th + 1) * np.abs(syf))
    wn, hn = f32(nw - 1), f32(nh - 1)
    G0 = np.maximum(wn * np.abs(sxf), hn * np.abs(syf))
    # the window's first pixel centre and the corner differences in float64
    dx0 = x_off + (ci + 0.5) * x_scale
    dy0 = y_off + (cj + 0.5) * y_scale
    (x0, y0), (x1, y1), (x2, y2), (x3, y3) = [(P[k, 0], P[k, 1]) for k in range(4)]
    # corners p0 (t0), p1 (t1), p2 (b0), p3 (b1); A = (p0; p1, p2), B = (p3; p2, p1)
    FA, stA = forms2(x0 - dx0, y0 - dy0, y0 - y2, x0 - x2, x0 - x1, y0 - y1, sxf, syf, XY2, G0, rng)
    FB, stB = forms2(x3 - dx0, y3 - dy0, y3 - y1, x3 - x1, x3 - x2, y3 - y2, sxf, syf, XY2, G0, rng)
    use = walk & (stA >= 0) & (stB >= 0) & ((stA | stB) != 0)
    # the test exercises the fast path: nearly every quad with a window takes it
    assert walk.mean() > 0.3 and use[walk].mean() > 0.99, (walk.mean(), use[walk].mean())
    K = K_LANE_WINDOW
    k = np.arange(K)[None, :]
    nwi = np.maximum(nw, 1).astype(np.int64)[:, None]
    kj, ki = k // nwi, k % nwi
    valid = use[:, None] & (k < cnt[:, None])
    codes = walk_codes(FA, FB, nwi, f32(ki), f32(kj))
    # the reference at the same pixels (absolute tile-local pixel indices)
    pi = ci[:, None] + ki
    pj = cj[:, None] + kj
    ref = ref_choice(P, x_off + (pi + 0.5) * x_scale, y_off + (pj + 0.5) * y_scale)
    bad = valid & (codes != 3) & (codes != ref)
    assert not bad.any(), (int(bad.sum()), np.argwhere(bad)[:5])
    unsure = (valid & (codes == 3)).sum() / max(valid.sum(), 1)
    assert unsure < (0.6 if adversarial else 0.002), unsure
    # T holds every pixel of the reference's window R the reference hits
    with np.errstate(invalid="ignore"):
        ri0 = np.floor((P[:, 0] - x_off) / x_scale).min(0)
        ri1 = np.floor((P[:, 0] - x_off) / x_scale).max(0)
        rj0 = np.floor((P[:, 1] - y_off) / y_scale).min(0)
        rj1 = np.floor((P[:, 1] - y_off) / y_scale).max(0)
    rw = ri1 - ri0 + 1
    rsel = use & (rw * (rj1 - rj0 + 1) <= 36)
    k36 = np.arange(36)[None, :]
    rwi = np.maximum(rw, 1).astype(np.int64)[:, None]
    rj, ri = rj0[:, None] + k36 // rwi, ri0[:, None] + k36 % rwi
    rvalid = rsel[:, None] & (k36 < (rw * (rj1 - rj0 + 1))[:, None])
    rref = ref_choice(P, x_off + (ri + 0.5) * x_scale, y_off + (rj + 0.5) * y_scale)
    inT = ((ri >= ci[:, None]) & (ri <= fi[:, None]) &
           (rj >= cj[:, None]) & (rj <= fj[:, None]))
    lost = rvalid & ~inT & (rref != 0)
    assert not lost.any(), (int(lost.sum()), np.argwhere(lost)[:5])
