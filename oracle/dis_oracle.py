"""CPU oracle of DIS optical flow -- TEST INFRASTRUCTURE ONLY (imported by tests/, never by neuralstyletransferv1_amd/).

The reference's default temporal flow (pipeline.py:1904-1914, --flow_method dis, run_videos.py:87 FLOW_METHOD):
    dis = cv2.DISOpticalFlow_create(cv2.DISOPTICAL_FLOW_PRESET_FAST); flow = dis.calc(prev_gray, gray, None)
OpenCV is not installed here (not importable, not in /root/reference), so this is a restatement of OpenCV's
DISOpticalFlowImpl (modules/video/src/dis_flow.cpp, Kroeger et al., "Fast Optical Flow using Dense Inverse
Search", ECCV 2016) and of its VariationalRefinement (variational_refinement.cpp, Brox et al. 2004 energy) with
PRESET_FAST's parameters: patch 8, stride 4, finest scale 2, 16 gradient-descent iterations, 5 variational
refinement iterations (alpha 20, gamma 10, delta 5, 5 SOR sweeps, omega 1.6, zeta 0.1, epsilon 0.001), mean
normalisation and spatial propagation on, border 16.  PARITY UNPINNED: nothing here is checked against cv2.

Restated per stage (per pyramid level, coarsest -> finest):
  pyramid          I0s/I1s by cv2.resize INTER_AREA (finest: rows / 2^s, then halving), I1 replicate-padded by
                   16, Sobel 3x3 gradients of I0 (spatialGradient, int16, BORDER_REFLECT_101)
  structure tensor separable running box sums of Ix^2, Iy^2, IxIy, Ix, Iy over every 8x8 patch (fp32, cv2's
                   running-sum order)
  inverse search   8 stripes of patch rows, each a forward and a backward sweep (8 + 8 inner iterations); per
                   patch: the flow at the patch centre (first sweep), the left / upper neighbour candidates
                   by mean-normalised SSD, then inverse-compositional Gauss-Newton steps with the inverted
                   structure tensor, stopping when the SSD stops falling; a result farther than 8 px from the
                   start is dropped
  densification    per pixel, the patches covering it weighted by 1 / max(1, |I1(x + u) - I0(x)|)
  variational      fixed-point iterations of the linearised Euler-Lagrange equations: data term (brightness
  refinement       and gradient constancy, normalised, robust weights), smoothness weights 10 / sqrt(|grad
                   (u + du)|^2 + |grad(v + dv)|^2 + eps^2) on the pixel grid, red-black SOR on (du, dv)
  upsampling       cv2.resize INTER_LINEAR to the next level, x 2; finally to the frame, x 2^finest
The 64-pixel patch sums run in the engine's order (a halving tree over the 64 pixels, row-major: the wave
reduction of dis_ops) instead of cv2's sequential / SIMD order, and the variational smoothness discretisation
(edge weights from forward differences, absent edges at the frame border) is this restatement's; everything
else follows cv2's operation order in fp32 (fp64 where cv2 uses double).
"""
from __future__ import annotations

import math

import numpy as np

from . import flow_oracle as FO

f32 = np.float32
PATCH, STRIDE, FINEST, GD_ITER, VR_ITER = 8, 4, 2, 16, 5
ALPHA, GAMMA, DELTA = 20.0, 10.0, 5.0
SOR_ITER, OMEGA, ZETA, EPSILON = 5, 1.6, 0.1, 0.001
BORDER = 16
NSTRIPES = 8
EPS = f32(0.001)
INF = f32(1e20)


def coarsest_scale(h: int, w: int) -> int:
    """dis_flow.cpp calc(): a search range of a quarter of the frame, a coarsest level >= one patch."""
    return min(int(math.log(max(w, h) / (4.0 * PATCH)) / math.log(2.0) + 0.5),
               int(math.log(min(w, h) / PATCH) / math.log(2.0)))


def sobel3(img: np.ndarray):
    """spatialGradient(I, dx, dy) (3x3 Sobel, BORDER_REFLECT_101) -> int16 dx, dy."""
    h, w = img.shape
    a = img.astype(np.int32)
    ys, xs = np.arange(h), np.arange(w)
    ym, yp = FO._refl101(ys - 1, h), FO._refl101(ys + 1, h)
    xm, xp = FO._refl101(xs - 1, w), FO._refl101(xs + 1, w)
    dxr = a[:, xp] - a[:, xm]
    dx = dxr[ym] + 2 * dxr + dxr[yp]
    dyr = a[yp] - a[ym]
    dy = dyr[:, xm] + 2 * dyr + dyr[:, xp]
    return dx.astype(np.int16), dy.astype(np.int16)


def structure_tensor(Ix: np.ndarray, Iy: np.ndarray, hs: int, ws: int):
    """precomputeStructureTensor: per patch (is, js) the fp32 box sums over its 8x8 pixels of Ix^2, Iy^2, IxIy,
    Ix, Iy, by cv2's running sums (horizontal: int products into fp32, then per stride; vertical over those)."""
    h, w = Ix.shape
    x, y = Ix.astype(np.int64), Iy.astype(np.int64)
    terms = [x * x, y * y, x * y, x, y]
    out = []
    for t in terms:
        aux = np.zeros((h, ws), f32)
        s = np.zeros(h, f32)
        for j in range(PATCH):
            s = (s + t[:, j].astype(f32)).astype(f32)
        aux[:, 0] = s
        js = 1
        for j in range(PATCH, w):
            s = (s + (t[:, j] - t[:, j - PATCH]).astype(f32)).astype(f32)
            if (j - PATCH + 1) % STRIDE == 0:
                if js < ws:
                    aux[:, js] = s
                js += 1
        res = np.zeros((hs, ws), f32)
        v = np.zeros(ws, f32)
        for i in range(PATCH):
            v = (v + aux[i]).astype(f32)
        res[0] = v
        is_ = 1
        for i in range(PATCH, h):
            v = (v + (aux[i] - aux[i - PATCH]).astype(f32)).astype(f32)
            if (i - PATCH + 1) % STRIDE == 0:
                if is_ < hs:
                    res[is_] = v
                is_ += 1
        out.append(res)
    return out  # xx, yy, xy, x, y


def _tree64(v: np.ndarray) -> np.ndarray:
    """Sum over the last axis (64 pixels, row-major) as the wave reduction adds them: a halving tree."""
    k = 32
    while k >= 1:
        v = (v[..., :k] + v[..., k:2 * k]).astype(f32)
        k //= 2
    return v[..., 0]


class _Level:
    def __init__(self, I0, I1):
        self.I0, self.I1 = I0, I1
        self.h, self.w = I0.shape
        self.I1e = np.pad(I1, BORDER, mode="edge")
        self.Ix, self.Iy = sobel3(I0)
        self.ws = 1 + (self.w - PATCH) // STRIDE
        self.hs = 1 + (self.h - PATCH) // STRIDE
        pi, pj = np.divmod(np.arange(64), 8)
        self.pi, self.pj = pi, pj

    def patch(self, arr, i, j):
        """[n] patch origins -> [n, 64] values of arr at the 8x8 pixels (row-major)."""
        return arr[i[:, None] + self.pi[None, :], j[:, None] + self.pj[None, :]]


def _bilinear_setup(L: _Level, i, j, ux, uy):
    """INIT_BILINEAR_WEIGHTS: clamped I1_ext coordinates of the patch origin + the 4 weights (fp32)."""
    il, iu = f32(BORDER - PATCH + 1), f32(BORDER + L.h - 1)
    jl, ju = f32(BORDER - PATCH + 1), f32(BORDER + L.w - 1)
    iI1 = np.minimum(np.maximum((i.astype(f32) + uy).astype(f32) + f32(BORDER), il), iu).astype(f32)
    jI1 = np.minimum(np.maximum((j.astype(f32) + ux).astype(f32) + f32(BORDER), jl), ju).astype(f32)
    di = (iI1 - np.floor(iI1)).astype(f32)
    dj = (jI1 - np.floor(jI1)).astype(f32)
    one = f32(1)
    w11 = (di * dj).astype(f32)
    w10 = (di * (one - dj)).astype(f32)
    w01 = ((one - di) * dj).astype(f32)
    w00 = ((one - di) * (one - dj)).astype(f32)
    return iI1.astype(np.int64), jI1.astype(np.int64), (w00, w01, w10, w11)


def _diffs(L: _Level, i, j, ux, uy):
    """[n,64] per-pixel diff = bilinear I1 - I0 (cv2's expression order)."""
    bi, bj, (w00, w01, w10, w11) = _bilinear_setup(L, i, j, ux, uy)
    a = L.patch(L.I1e, bi, bj).astype(f32)
    b = L.patch(L.I1e, bi, bj + 1).astype(f32)
    c = L.patch(L.I1e, bi + 1, bj).astype(f32)
    d = L.patch(L.I1e, bi + 1, bj + 1).astype(f32)
    t = (w00[:, None] * a).astype(f32)
    t = (t + (w01[:, None] * b).astype(f32)).astype(f32)
    t = (t + (w10[:, None] * c).astype(f32)).astype(f32)
    t = (t + (w11[:, None] * d).astype(f32)).astype(f32)
    return (t - L.patch(L.I0, i, j).astype(f32)).astype(f32)


def _ssd_mean_norm(L, i, j, ux, uy):
    diff = _diffs(L, i, j, ux, uy)
    sd = _tree64(diff)
    sq = _tree64((diff * diff).astype(f32))
    n = f32(64)
    return (sq - ((sd * sd).astype(f32) / n).astype(f32)).astype(f32)


def inverse_search(L: _Level, Ux: np.ndarray, Uy: np.ndarray, tensor):
    """PatchInverseSearch_ParBody over NSTRIPES stripes with spatial propagation (num_iter 2): -> Sx, Sy [hs,ws]."""
    hs, ws = L.hs, L.ws
    xx, yy, xy, gx, gy = tensor
    Sx = np.zeros((hs, ws), f32)
    Sy = np.zeros((hs, ws), f32)
    stripe = int(math.ceil(hs / NSTRIPES))
    inner = int(math.floor(GD_ITER / 2.0))
    n64 = f32(64)
    for it in range(2):
        fwd = it % 2 == 0
        # every stripe's rows; a step processes the patches on one anti-diagonal of every stripe (the patch
        # (is, js) depends only on its left / upper (forward) or right / lower (backward) neighbour)
        nstep = ws + stripe - 1
        for t in range(nstep):
            iss, jss, first_row, first_col = [], [], [], []
            for s in range(NSTRIPES):
                r0, r1 = min(s * stripe, hs), min((s + 1) * stripe, hs)
                for r in range(r1 - r0):
                    c = t - r
                    if not (0 <= c < ws):
                        continue
                    if fwd:
                        iss.append(r0 + r)
                        jss.append(c)
                    else:
                        iss.append(r1 - 1 - r)
                        jss.append(ws - 1 - c)
                    first_row.append(r == 0)
                    first_col.append(c == 0)
            if not iss:
                continue
            is_ = np.array(iss)
            js = np.array(jss)
            i = is_ * STRIDE
            j = js * STRIDE
            if it == 0:
                Sx[is_, js] = Ux[i + PATCH // 2, j + PATCH // 2]
                Sy[is_, js] = Uy[i + PATCH // 2, j + PATCH // 2]
            cx, cy = Sx[is_, js].copy(), Sy[is_, js].copy()
            min_ssd = _ssd_mean_norm(L, i, j, cx, cy)
            d = 1 if fwd else -1
            # left (forward) / right (backward) neighbour in the row
            has = ~np.array(first_col)
            if has.any():
                nx, ny = Sx[is_, np.clip(js - d, 0, ws - 1)], Sy[is_, np.clip(js - d, 0, ws - 1)]
                cs = _ssd_mean_norm(L, i, j, nx, ny)
                take = has & (cs < min_ssd)
                min_ssd = np.where(take, cs, min_ssd)
                cx, cy = np.where(take, nx, cx), np.where(take, ny, cy)
            # upper (forward) / lower (backward) neighbour in the stripe
            has = ~np.array(first_row)
            if has.any():
                nx, ny = Sx[np.clip(is_ - d, 0, hs - 1), js], Sy[np.clip(is_ - d, 0, hs - 1), js]
                cs = _ssd_mean_norm(L, i, j, nx, ny)
                take = has & (cs < min_ssd)
                min_ssd = np.where(take, cs, min_ssd)
                cx, cy = np.where(take, nx, cx), np.where(take, ny, cy)
            Sx[is_, js], Sy[is_, js] = cx, cy
            # inverse-compositional Gauss-Newton steps
            a, b, c2 = xx[is_, js], yy[is_, js], xy[is_, js]
            det = ((a * b).astype(f32) - (c2 * c2).astype(f32)).astype(f32)
            det = np.where(np.abs(det) < EPS, EPS, det).astype(f32)
            h11 = (b / det).astype(f32)
            h12 = (-c2 / det).astype(f32)
            h22 = (a / det).astype(f32)
            xs, ys = gx[is_, js], gy[is_, js]
            I0x = L.patch(L.Ix, i, j).astype(f32)
            I0y = L.patch(L.Iy, i, j).astype(f32)
            ux, uy = cx.copy(), cy.copy()
            prev = np.full(len(is_), INF, f32)
            active = np.ones(len(is_), bool)
            for _ in range(inner):
                diff = _diffs(L, i, j, ux, uy)
                sd = _tree64(diff)
                sq = _tree64((diff * diff).astype(f32))
                sxm = _tree64((diff * I0x).astype(f32))
                sym = _tree64((diff * I0y).astype(f32))
                dux = (sxm - ((sd * xs).astype(f32) / n64).astype(f32)).astype(f32)
                duy = (sym - ((sd * ys).astype(f32) / n64).astype(f32)).astype(f32)
                ssd = (sq - ((sd * sd).astype(f32) / n64).astype(f32)).astype(f32)
                dx = ((h11 * dux).astype(f32) + (h12 * duy).astype(f32)).astype(f32)
                dy = ((h12 * dux).astype(f32) + (h22 * duy).astype(f32)).astype(f32)
                ux = np.where(active, (ux - dx).astype(f32), ux)
                uy = np.where(active, (uy - dy).astype(f32), uy)
                active = active & ~(ssd >= prev)
                prev = np.where(active, ssd, prev)
                if not active.any():
                    break
            # norm(Vec2f(cur - start)): fp32 differences, squared and summed in double
            ex = (ux - cx).astype(f32).astype(np.float64)
            ey = (uy - cy).astype(f32).astype(np.float64)
            keep = np.sqrt(ex * ex + ey * ey) <= PATCH
            Sx[is_, js] = np.where(keep, ux, cx)
            Sy[is_, js] = np.where(keep, uy, cy)
    return Sx, Sy


def densify(L: _Level, Sx: np.ndarray, Sy: np.ndarray):
    """Densification_ParBody: per pixel the patches overlapping it (in is, js order)."""
    h, w, hs, ws = L.h, L.w, L.hs, L.ws

    def ranges(n, ns):
        lo = np.zeros(n, np.int64)
        hi = np.zeros(n, np.int64)
        s, e = 0, -1
        for i in range(n):
            if i % STRIDE == 0 and i + PATCH <= n:
                e += 1
            if i - PATCH >= 0 and (i - PATCH) % STRIDE == 0 and s < e:
                s += 1
            lo[i], hi[i] = s, e
        return lo, hi
    ilo, ihi = ranges(h, hs)
    jlo, jhi = ranges(w, ws)
    ys, xs = np.mgrid[0:h, 0:w]
    I1 = L.I1.astype(f32)
    I0 = L.I0.astype(f32)
    sux = np.zeros((h, w), f32)
    suy = np.zeros((h, w), f32)
    sc = np.zeros((h, w), f32)
    wm1, hm1 = f32(w - 1.0) - EPS, f32(h - 1.0) - EPS
    for a in range(3):
        for b in range(3):
            is_ = ilo[ys] + a
            js = jlo[xs] + b
            ok = (is_ <= ihi[ys]) & (js <= jhi[xs])
            isc, jsc = np.minimum(is_, hs - 1), np.minimum(js, ws - 1)
            sx, sy = Sx[isc, jsc], Sy[isc, jsc]
            jm = np.minimum(np.maximum((xs.astype(f32) + sx).astype(f32), f32(0)), wm1).astype(f32)
            im = np.minimum(np.maximum((ys.astype(f32) + sy).astype(f32), f32(0)), hm1).astype(f32)
            jl, il = jm.astype(np.int64), im.astype(np.int64)
            ju, iu = jl + 1, il + 1
            jlf, ilf, juf, iuf = jl.astype(f32), il.astype(f32), ju.astype(f32), iu.astype(f32)
            t = (((jm - jlf) * (im - ilf)).astype(f32) * I1[iu, ju]).astype(f32)
            t = (t + (((juf - jm) * (im - ilf)).astype(f32) * I1[iu, jl]).astype(f32)).astype(f32)
            t = (t + (((jm - jlf) * (iuf - im)).astype(f32) * I1[il, ju]).astype(f32)).astype(f32)
            t = (t + (((juf - jm) * (iuf - im)).astype(f32) * I1[il, jl]).astype(f32)).astype(f32)
            diff = (t - I0).astype(f32)
            coef = (f32(1) / np.maximum(f32(1), np.abs(diff))).astype(f32)
            sux = np.where(ok, (sux + (coef * sx).astype(f32)).astype(f32), sux)
            suy = np.where(ok, (suy + (coef * sy).astype(f32)).astype(f32), suy)
            sc = np.where(ok, (sc + coef).astype(f32), sc)
    return (sux / sc).astype(f32), (suy / sc).astype(f32)


def _remap_rep(img: np.ndarray, mx: np.ndarray, my: np.ndarray) -> np.ndarray:
    """cv2.remap(img, mx, my, INTER_LINEAR, BORDER_REPLICATE) of a float image (1/32-pixel fixed point)."""
    h, w = img.shape
    mx = np.clip(np.nan_to_num(mx, nan=-2.0 * w), -2.0 * w, 3.0 * w).astype(f32)
    my = np.clip(np.nan_to_num(my, nan=-2.0 * h), -2.0 * h, 3.0 * h).astype(f32)
    X = np.rint(mx * f32(32)).astype(np.int64)
    Y = np.rint(my * f32(32)).astype(np.int64)
    sx, sy = X >> 5, Y >> 5
    fx = (X & 31).astype(f32) * f32(1 / 32)
    fy = (Y & 31).astype(f32) * f32(1 / 32)
    one = f32(1)
    x0, x1 = np.clip(sx, 0, w - 1), np.clip(sx + 1, 0, w - 1)
    y0, y1 = np.clip(sy, 0, h - 1), np.clip(sy + 1, 0, h - 1)
    t0 = (img[y0, x0] * ((one - fy) * (one - fx))).astype(f32) + (img[y0, x1] * ((one - fy) * fx)).astype(f32)
    t1 = (img[y1, x0] * (fy * (one - fx))).astype(f32) + (img[y1, x1] * (fy * fx)).astype(f32)
    return (t0.astype(f32) + t1.astype(f32)).astype(f32)


def _dx(a):  # Sobel ksize 1: I(x+1) - I(x-1), BORDER_REPLICATE
    w = a.shape[1]
    xs = np.arange(w)
    return (a[:, np.minimum(xs + 1, w - 1)] - a[:, np.maximum(xs - 1, 0)]).astype(f32)


def _dy(a):
    h = a.shape[0]
    ys = np.arange(h)
    return (a[np.minimum(ys + 1, h - 1)] - a[np.maximum(ys - 1, 0)]).astype(f32)


def variational_refinement(I0: np.ndarray, I1: np.ndarray, U: np.ndarray, V: np.ndarray):
    """VariationalRefinement.calcUV (FAST: 5 fixed-point iterations x 5 red-black SOR sweeps) -> U + dU, V + dV."""
    h, w = I0.shape
    zeta2 = f32(ZETA * ZETA)
    eps2 = f32(EPSILON * EPSILON)
    alpha2, gamma2, delta2 = f32(ALPHA / 2), f32(GAMMA / 2), f32(DELTA / 2)
    omega = f32(OMEGA)
    ys, xs = np.mgrid[0:h, 0:w]
    I0f, I1f = I0.astype(f32), I1.astype(f32)
    I1w = _remap_rep(I1f, (xs.astype(f32) + U).astype(f32), (ys.astype(f32) + V).astype(f32))
    avg = ((f32(0.5) * I0f).astype(f32) + (f32(0.5) * I1w).astype(f32)).astype(f32)
    Iz = (I1w - I0f).astype(f32)
    Ix, Iy = _dx(avg), _dy(avg)
    Ixz, Iyz = _dx(Iz), _dy(Iz)
    Ixx, Ixy, Iyy = _dx(Ix), _dy(Ix), _dy(Iy)
    dU = np.zeros((h, w), f32)
    dV = np.zeros((h, w), f32)
    red = ((ys + xs) % 2) == 0
    hasR, hasL = xs < w - 1, xs > 0
    hasD, hasU = ys < h - 1, ys > 0

    def sh(a, dy, dx):  # a[y + dy, x + dx] clamped (only read where the neighbour exists)
        return a[np.clip(ys + dy, 0, h - 1), np.clip(xs + dx, 0, w - 1)]

    for _ in range(VR_ITER):
        # data term (ComputeDataTerm_ParBody)
        dn = ((Ix * Ix).astype(f32) + (Iy * Iy).astype(f32) + zeta2).astype(f32)
        k = (Iz + (Ix * dU).astype(f32) + (Iy * dV).astype(f32)).astype(f32)
        wt = ((delta2 / np.sqrt(((k * k).astype(f32) / dn).astype(f32) + eps2).astype(f32)).astype(f32) / dn).astype(f32)
        a11 = ((wt * (Ix * Ix).astype(f32)).astype(f32) + zeta2).astype(f32)
        a12 = (wt * (Ix * Iy).astype(f32)).astype(f32)
        a22 = ((wt * (Iy * Iy).astype(f32)).astype(f32) + zeta2).astype(f32)
        b1 = (-wt * (Iz * Ix).astype(f32)).astype(f32)
        b2 = (-wt * (Iz * Iy).astype(f32)).astype(f32)
        dn1 = ((Ixx * Ixx).astype(f32) + (Ixy * Ixy).astype(f32) + zeta2).astype(f32)
        dn2 = ((Iyy * Iyy).astype(f32) + (Ixy * Ixy).astype(f32) + zeta2).astype(f32)
        kx = (Ixz + (Ixx * dU).astype(f32) + (Ixy * dV).astype(f32)).astype(f32)
        ky = (Iyz + (Ixy * dU).astype(f32) + (Iyy * dV).astype(f32)).astype(f32)
        wt = (gamma2 / np.sqrt((((kx * kx).astype(f32) / dn1).astype(f32) + ((ky * ky).astype(f32) / dn2).astype(f32)
                                + eps2).astype(f32)).astype(f32)).astype(f32)

        def g(p, q, r, s):  # p*q/dn1 + r*s/dn2
            return ((((p * q).astype(f32) / dn1).astype(f32) + ((r * s).astype(f32) / dn2).astype(f32))).astype(f32)
        a11 = (a11 + (wt * g(Ixx, Ixx, Ixy, Ixy)).astype(f32)).astype(f32)
        a12 = (a12 + (wt * g(Ixx, Ixy, Ixy, Iyy)).astype(f32)).astype(f32)
        a22 = (a22 + (wt * g(Ixy, Ixy, Iyy, Iyy)).astype(f32)).astype(f32)
        b1 = (b1 + (-wt * g(Ixx, Ixz, Ixy, Iyz)).astype(f32)).astype(f32)
        b2 = (b2 + (-wt * g(Ixy, Ixz, Iyy, Iyz)).astype(f32)).astype(f32)
        # smoothness weights of the current flow U + dU (forward differences; 0 past the last row / column)
        tU = (U + dU).astype(f32)
        tV = (V + dV).astype(f32)
        ux = np.where(hasR, (sh(tU, 0, 1) - tU).astype(f32), f32(0))
        vx = np.where(hasR, (sh(tV, 0, 1) - tV).astype(f32), f32(0))
        uy = np.where(hasD, (sh(tU, 1, 0) - tU).astype(f32), f32(0))
        vy = np.where(hasD, (sh(tV, 1, 0) - tV).astype(f32), f32(0))
        s2 = ((ux * ux).astype(f32) + (vx * vx).astype(f32) + (uy * uy).astype(f32) + (vy * vy).astype(f32)
              + eps2).astype(f32)
        phi = (alpha2 / np.sqrt(s2).astype(f32)).astype(f32)
        # edge weights: right / down edges carry the pixel's own weight, left / up its neighbour's
        wR = np.where(hasR, phi, f32(0))
        wL = np.where(hasL, sh(phi, 0, -1), f32(0))
        wD = np.where(hasD, phi, f32(0))
        wUp = np.where(hasU, sh(phi, -1, 0), f32(0))
        edges = [(wL, 0, -1), (wR, 0, 1), (wUp, -1, 0), (wD, 1, 0)]
        for (we, dy, dx) in edges:
            a11 = (a11 + we).astype(f32)
            a22 = (a22 + we).astype(f32)
            b1 = (b1 + (we * (sh(U, dy, dx) - U).astype(f32)).astype(f32)).astype(f32)
            b2 = (b2 + (we * (sh(V, dy, dx) - V).astype(f32)).astype(f32)).astype(f32)
        # red-black SOR on (dU, dV)
        for _s in range(SOR_ITER):
            for color in (red, ~red):
                su = np.zeros((h, w), f32)
                sv = np.zeros((h, w), f32)
                for (we, dy, dx) in edges:
                    su = (su + (we * sh(dU, dy, dx)).astype(f32)).astype(f32)
                    sv = (sv + (we * sh(dV, dy, dx)).astype(f32)).astype(f32)
                nu = (dU + (omega * (((su + b1 - (dV * a12).astype(f32)).astype(f32) / a11).astype(f32) - dU)
                            .astype(f32)).astype(f32)).astype(f32)
                dU = np.where(color, nu, dU)
                nv = (dV + (omega * (((sv + b2 - (dU * a12).astype(f32)).astype(f32) / a22).astype(f32) - dV)
                            .astype(f32)).astype(f32)).astype(f32)
                dV = np.where(color, nv, dV)
    return (U + dU).astype(f32), (V + dV).astype(f32)


def dis_flow(prev: np.ndarray, nxt: np.ndarray, vr_iter: int = VR_ITER) -> np.ndarray:
    """cv2.DISOpticalFlow_create(PRESET_FAST).calc(prev, nxt, None) restated: u8 [h,w] x 2 -> flow [h,w,2] f32."""
    H, W = prev.shape
    cs = coarsest_scale(H, W)
    if cs < FINEST:
        raise ValueError(f"frame {W}x{H} too small for DIS PRESET_FAST (coarsest scale {cs} < finest {FINEST})")
    I0s, I1s = {}, {}
    for s in range(FINEST, cs + 1):
        if s == FINEST:
            rows, cols = H // (1 << s), W // (1 << s)
            I0s[s], I1s[s] = FO.area_resize(prev, rows, cols), FO.area_resize(nxt, rows, cols)
        else:
            rows, cols = I0s[s - 1].shape[0] // 2, I0s[s - 1].shape[1] // 2
            I0s[s], I1s[s] = FO.area_resize(I0s[s - 1], rows, cols), FO.area_resize(I1s[s - 1], rows, cols)
    Ux = np.zeros(I0s[cs].shape, f32)
    Uy = np.zeros(I0s[cs].shape, f32)
    for s in range(cs, FINEST - 1, -1):
        L = _Level(I0s[s], I1s[s])
        tensor = structure_tensor(L.Ix, L.Iy, L.hs, L.ws)
        Sx, Sy = inverse_search(L, Ux, Uy, tensor)
        Ux, Uy = densify(L, Sx, Sy)
        if vr_iter > 0:
            Ux, Uy = variational_refinement(L.I0, L.I1, Ux, Uy)
        if s > FINEST:
            h1, w1 = I0s[s - 1].shape
            Ux = FO.resize_lin(Ux, h1, w1, 2.0)
            Uy = FO.resize_lin(Uy, h1, w1, 2.0)
    U = np.stack([Ux, Uy], axis=-1)
    return FO.resize_lin(U, H, W, float(1 << FINEST))
