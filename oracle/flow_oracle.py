"""CPU oracle of the temporal stage (--flow_ema / --motion_blend, pipeline.py:1884-1940, 2072-2086) -- TEST
INFRASTRUCTURE ONLY (imported by tests/, never by neuralstyletransferv1_amd/).

  gray          pil_rgb.convert("L") -- Pillow itself (the reference's call, pinned)
  farneback     cv2.calcOpticalFlowFarneback(prev, next, None, 0.5, 3, 15, 3, 5, 1.1, 0) restated in numpy after
                OpenCV's optflowgf.cpp (FarnebackPrepareGaussian / PolyExp / UpdateMatrices / UpdateFlow_Blur and
                the pyramid loop of calcOpticalFlowFarneback), with the engine's operation order
  fuse          the flow EMA with _warp_with_flow's cv2.remap(INTER_LINEAR, BORDER_REPLICATE) restated
  motion_alpha  clip(|flow| / 8) -> cv2.GaussianBlur(sigma 3) restated -> blend - (blend - 0.4) * m
cv2 is not installed here, so everything but `gray` is PARITY UNPINNED: the restatement is checked against the
GPU and against properties (a translated texture yields its translation).
"""
from __future__ import annotations

import math

import numpy as np
from PIL import Image

f32 = np.float32


def gray(rgb_u8: np.ndarray) -> np.ndarray:
    return np.array(Image.fromarray(rgb_u8, mode="RGB").convert("L"), dtype=np.uint8)


def gaussian_taps(n: int, sigma: float) -> np.ndarray:
    """cv2.getGaussianKernel(n, sigma, CV_32F) (the fixed 3-tap table when sigma <= 0)."""
    if sigma <= 0 and n == 3:
        return np.array([0.25, 0.5, 0.25], dtype=f32)
    if sigma <= 0:
        sigma = ((n - 1) * 0.5 - 1) * 0.3 + 0.8
    s2 = -0.5 / (sigma * sigma)
    v = [math.exp(s2 * (i - (n - 1) * 0.5) ** 2) for i in range(n)]
    s = sum(v)
    return np.array([x / s for x in v], dtype=f32)


def _refl101(p: np.ndarray, n: int) -> np.ndarray:
    p = np.abs(p)
    return np.where(p >= n, 2 * n - 2 - p, p)


def gauss_blur(img: np.ndarray, ksize: int, sigma: float) -> np.ndarray:
    t = gaussian_taps(ksize, sigma)
    h, w = img.shape
    r = ksize // 2
    xs, ys = np.arange(w), np.arange(h)
    acc = np.zeros_like(img, dtype=f32)
    for j in range(ksize):
        acc = acc + t[j] * img[:, _refl101(xs + j - r, w)]
    out = np.zeros_like(acc)
    for j in range(ksize):
        out = out + t[j] * acc[_refl101(ys + j - r, h), :]
    return out


def _coef(n_out: int, n_in: int):
    scale = n_in / n_out
    d = np.arange(n_out)
    f = ((d + 0.5) * scale - 0.5).astype(f32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(f32)).astype(f32)
    lo = s < 0
    f[lo], s[lo] = 0, 0
    hi = s >= n_in - 1
    f[hi], s[hi] = 0, n_in - 1
    return s, f


def resize_lin(img: np.ndarray, oh: int, ow: int, mul: float = 1.0) -> np.ndarray:
    """cv2.resize INTER_LINEAR of [h,w] or [h,w,c] float32 (then * mul)."""
    h, w = img.shape[:2]
    sx, fx = _coef(ow, w)
    sy, fy = _coef(oh, h)
    x1, y1 = np.minimum(sx + 1, w - 1), np.minimum(sy + 1, h - 1)
    if img.ndim == 3:
        fx, fy = fx[None, :, None], fy[:, None, None]
    else:
        fx, fy = fx[None, :], fy[:, None]
    one = f32(1)
    r0 = img[sy][:, sx] * (one - fx) + img[sy][:, x1] * fx
    r1 = img[y1][:, sx] * (one - fx) + img[y1][:, x1] * fx
    return ((r0 * (one - fy) + r1 * fy) * f32(mul)).astype(f32)


def poly_tab(n: int, sigma: float):
    if sigma < 1.19209290e-07:
        sigma = n * 0.3
    g = np.zeros(2 * n + 1, dtype=f32)
    s = 0.0
    for x in range(-n, n + 1):
        g[x + n] = f32(math.exp(-x * x / (2 * sigma * sigma)))
        s += float(g[x + n])
    s = 1.0 / s
    xg, xxg = np.zeros_like(g), np.zeros_like(g)
    for x in range(-n, n + 1):
        g[x + n] = f32(float(g[x + n]) * s)
        xg[x + n] = f32(x) * g[x + n]
        xxg[x + n] = f32(x * x) * g[x + n]
    gd = g.astype(np.float64)
    G00 = G11 = G33 = G55 = 0.0
    for y in range(-n, n + 1):
        for x in range(-n, n + 1):
            G00 += gd[y + n] * gd[x + n]
            G11 += gd[y + n] * gd[x + n] * x * x
            G33 += gd[y + n] * gd[x + n] * x * x * x * x
            G55 += gd[y + n] * gd[x + n] * x * x * y * y
    a, b, c, d = G00, G11, G33, G55
    det = a * (c * c - d * d) - b * (b * c - b * d) + b * (b * d - c * b)
    return g, xg, xxg, 1.0 / b, -(b * c - b * d) / det, (a * c - b * b) / det, 1.0 / d


def poly_exp(src: np.ndarray, n: int, sigma: float) -> np.ndarray:
    g, xg, xxg, ig11, ig03, ig33, ig55 = poly_tab(n, sigma)
    h, w = src.shape
    ys = np.arange(h)
    t0 = src * g[n]
    t1 = np.zeros_like(src)
    t2 = np.zeros_like(src)
    for k in range(1, n + 1):
        a = src[np.maximum(ys - k, 0)]
        b = src[np.minimum(ys + k, h - 1)]
        p = a + b
        t0 = t0 + g[n + k] * p
        t1 = t1 + xg[n + k] * (b - a)
        t2 = t2 + xxg[n + k] * p
    xs = np.arange(w)
    b1 = (t0 * g[n]).astype(np.float64)
    b3 = (t1 * g[n]).astype(np.float64)
    b5 = (t2 * g[n]).astype(np.float64)
    b2 = np.zeros((h, w))
    b4 = np.zeros((h, w))
    b6 = np.zeros((h, w))
    for k in range(1, n + 1):
        xp, xm = np.minimum(xs + k, w - 1), np.maximum(xs - k, 0)
        tg = (t0[:, xp] + t0[:, xm]).astype(np.float64)
        b1 += tg * float(g[n + k])
        b4 += tg * float(xxg[n + k])
        b2 += ((t0[:, xp] - t0[:, xm]) * xg[n + k]).astype(np.float64)
        b3 += ((t1[:, xp] + t1[:, xm]) * g[n + k]).astype(np.float64)
        b6 += ((t1[:, xp] - t1[:, xm]) * xg[n + k]).astype(np.float64)
        b5 += ((t2[:, xp] + t2[:, xm]) * g[n + k]).astype(np.float64)
    R = np.zeros((h, w, 5), dtype=f32)
    R[..., 1] = b2 * ig11
    R[..., 0] = b3 * ig11
    R[..., 3] = b1 * ig03 + b4 * ig33
    R[..., 2] = b1 * ig03 + b5 * ig33
    R[..., 4] = b6 * ig55
    return R


def update_matrices(R0: np.ndarray, R1: np.ndarray, flow: np.ndarray) -> np.ndarray:
    h, w, _ = R0.shape
    border = np.array([0.14, 0.14, 0.4472, 0.4472, 0.4472], dtype=f32)
    ys, xs = np.mgrid[0:h, 0:w]
    dx, dy = flow[..., 0], flow[..., 1]
    fx = xs.astype(f32) + dx
    fy = ys.astype(f32) + dy
    x1 = np.floor(fx).astype(np.int64)
    y1 = np.floor(fy).astype(np.int64)
    fx = fx - x1.astype(f32)
    fy = fy - y1.astype(f32)
    inside = (x1 >= 0) & (x1 < w - 1) & (y1 >= 0) & (y1 < h - 1)
    xc, yc = np.clip(x1, 0, w - 2), np.clip(y1, 0, h - 2)
    one = f32(1)
    a00, a01, a10, a11 = (one - fx) * (one - fy), fx * (one - fy), (one - fx) * fy, fx * fy
    v = [a00 * R1[yc, xc, c] + a01 * R1[yc, xc + 1, c] + a10 * R1[yc + 1, xc, c] + a11 * R1[yc + 1, xc + 1, c]
         for c in range(5)]
    r2 = np.where(inside, v[0], f32(0))
    r3 = np.where(inside, v[1], f32(0))
    r4 = np.where(inside, (R0[..., 2] + v[2]) * f32(0.5), R0[..., 2])
    r5 = np.where(inside, (R0[..., 3] + v[3]) * f32(0.5), R0[..., 3])
    r6 = np.where(inside, (R0[..., 4] + v[4]) * f32(0.25), R0[..., 4] * f32(0.5))
    r2 = (R0[..., 0] - r2) * f32(0.5)
    r3 = (R0[..., 1] - r3) * f32(0.5)
    r2 = r2 + (r4 * dy + r6 * dx)
    r3 = r3 + (r6 * dy + r5 * dx)
    bx0 = np.where(xs < 5, border[np.minimum(xs, 4)], one)
    bx1 = np.where(xs >= w - 5, border[np.clip(w - xs - 1, 0, 4)], one)
    by0 = np.where(ys < 5, border[np.minimum(ys, 4)], one)
    by1 = np.where(ys >= h - 5, border[np.clip(h - ys - 1, 0, 4)], one)
    edge = (xs < 5) | (xs >= w - 5) | (ys < 5) | (ys >= h - 5)
    sc = np.where(edge, ((bx0 * bx1) * by0) * by1, one).astype(f32)
    r2, r3, r4, r5, r6 = (np.where(edge, r * sc, r) for r in (r2, r3, r4, r5, r6))
    M = np.zeros((h, w, 5), dtype=f32)
    M[..., 0] = r4 * r4 + r6 * r6
    M[..., 1] = (r4 + r5) * r6
    M[..., 2] = r5 * r5 + r6 * r6
    M[..., 3] = r4 * r2 + r6 * r3
    M[..., 4] = r6 * r2 + r5 * r3
    return M


def blur_solve(M: np.ndarray, winsize: int) -> np.ndarray:
    h, w, _ = M.shape
    m = winsize // 2
    ys, xs = np.arange(h), np.arange(w)
    # running vertical sums per strip of 16 rows as the engine (and OpenCV) keeps them: the first window summed,
    # then + (entering - leaving) with the row difference in float
    vs = np.zeros((h, w, 5))
    for y0 in range(0, h, 16):
        s = np.zeros((w, 5))
        for q in range(y0 - m, y0 + m + 1):
            s = s + M[min(max(q, 0), h - 1)].astype(np.float64)
        for y in range(y0, min(h, y0 + 16)):
            if y > y0:
                s = s + (M[min(y + m, h - 1)] - M[max(y - m - 1, 0)]).astype(np.float64)
            vs[y] = s
    s = np.zeros((h, w, 5))
    for q in range(-m, m + 1):
        s += vs[:, np.clip(xs + q, 0, w - 1)]
    sc = 1.0 / (winsize * winsize)
    g11, g12, g22, h1, h2 = (s[..., c] * sc for c in range(5))
    idet = 1.0 / (g11 * g22 - g12 * g12 + 1e-3)
    return np.stack([(g11 * h2 - g12 * h1) * idet, (g22 * h1 - g12 * h2) * idet], -1).astype(f32)


def farneback(prev: np.ndarray, nxt: np.ndarray, pyr_scale=0.5, levels=3, winsize=15, iterations=3, poly_n=5,
              poly_sigma=1.1) -> np.ndarray:
    h, w = prev.shape
    scale, k = 1.0, 0
    while k < levels:
        scale *= pyr_scale
        if w * scale < 32 or h * scale < 32:
            break
        k += 1
    levels = k
    prev_flow = None
    for k in range(levels, -1, -1):
        scale = 1.0
        for _ in range(k):
            scale *= pyr_scale
        sigma = (1.0 / scale - 1) * 0.5
        ksz = max(int(np.rint(sigma * 5)) | 1, 3)
        lw, lh = int(np.rint(w * scale)), int(np.rint(h * scale))
        flow = (np.zeros((lh, lw, 2), dtype=f32) if prev_flow is None
                else resize_lin(prev_flow, lh, lw, 1.0 / pyr_scale))
        R = []
        for img in (prev, nxt):
            b = gauss_blur(img.astype(f32), ksz, sigma)
            if (lh, lw) != (h, w):
                b = resize_lin(b, lh, lw)
            R.append(poly_exp(b, poly_n, poly_sigma))
        M = update_matrices(R[0], R[1], flow)
        for it in range(iterations):
            flow = blur_solve(M, winsize)
            if it < iterations - 1:
                M = update_matrices(R[0], R[1], flow)
        prev_flow = flow
    return prev_flow


def fuse(curr01: np.ndarray, prev01: np.ndarray, flow: np.ndarray, a: float) -> np.ndarray:
    """[3,h,w] planes; remap BORDER_REPLICATE in OpenCV's 1/32-pixel fixed point."""
    _, h, w = curr01.shape
    ys, xs = np.mgrid[0:h, 0:w]
    mx = np.clip(np.nan_to_num(xs.astype(f32) + flow[..., 0], nan=-2.0 * w), -2.0 * w, 3.0 * w).astype(f32)
    my = np.clip(np.nan_to_num(ys.astype(f32) + flow[..., 1], nan=-2.0 * h), -2.0 * h, 3.0 * h).astype(f32)
    X = np.rint(mx * f32(32)).astype(np.int64)
    Y = np.rint(my * f32(32)).astype(np.int64)
    sx, sy = X >> 5, Y >> 5
    fx = (X & 31).astype(f32) * f32(1 / 32)
    fy = (Y & 31).astype(f32) * f32(1 / 32)
    one = f32(1)
    x0, x1 = np.clip(sx, 0, w - 1), np.clip(sx + 1, 0, w - 1)
    y0, y1 = np.clip(sy, 0, h - 1), np.clip(sy + 1, 0, h - 1)
    out = np.empty_like(curr01)
    for c in range(3):
        p = prev01[c]
        t0 = p[y0, x0] * ((one - fy) * (one - fx)) + p[y0, x1] * ((one - fy) * fx)
        t1 = p[y1, x0] * (fy * (one - fx)) + p[y1, x1] * (fy * fx)
        out[c] = np.clip(f32(a) * curr01[c] + f32(1.0 - a) * (t0 + t1), 0, 1)
    return out


def motion_alpha(flow: np.ndarray, blend: float) -> np.ndarray:
    mag = np.sqrt(flow[..., 0] ** 2 + flow[..., 1] ** 2).astype(f32)
    m = np.clip(mag / f32(8.0), 0, 1)
    m = gauss_blur(m, int(np.rint(3.0 * 8 + 1)) | 1, 3.0)
    return (f32(blend) - f32(blend - 0.4) * m).astype(f32)


def _area_cells(ssize: int, dsize: int, scale: float):
    """computeResizeAreaTab (OpenCV resize.cpp) for one axis: per destination index the (source, weight) cells,
    weights the fp32 of the double ratios; partial first / last cells only beyond 1e-3."""
    cells = []
    for d in range(dsize):
        fs1 = d * scale
        fs2 = fs1 + scale
        cell = min(scale, ssize - fs1)
        s1, s2 = math.ceil(fs1), math.floor(fs2)
        s2 = min(s2, ssize - 1)
        s1 = min(s1, s2)
        row = []
        if s1 - fs1 > 1e-3:
            row.append((s1 - 1, f32((s1 - fs1) / cell)))
        for sx in range(s1, s2):
            row.append((sx, f32(1.0 / cell)))
        if fs2 - s2 > 1e-3:
            row.append((s2, f32(min(min(fs2 - s2, 1.0), cell) / cell)))
        cells.append(row)
    return cells


def area_resize(img: np.ndarray, oh: int, ow: int) -> np.ndarray:
    """cv2.resize(img, (ow, oh), interpolation=INTER_AREA) of a u8 image [h,w] or [h,w,c], downscaling (OpenCV
    resize.cpp restated: integer scales -> resizeAreaFast_ (int block sum * fp32 1/area, cvRound; scale 2 x 2
    -> ResizeAreaFastVec's (sum + 2) >> 2, rounding halves up), else ResizeArea_Invoker over computeResizeAreaTab's cells: per
    source row buf = sum(S * alpha) in cell order, sum = beta * buf, then += beta * buf; cvRound + saturate)."""
    h, w = img.shape[:2]
    sx, sy = 1.0 / (ow / w), 1.0 / (oh / h)
    isx, isy = int(round(sx)), int(round(sy))
    x = img.reshape(h, w, -1)
    if abs(sx - isx) < np.finfo(np.float64).eps and abs(sy - isy) < np.finfo(np.float64).eps:
        s = x[:oh * isy, :ow * isx].reshape(oh, isy, ow, isx, -1).astype(np.int64).sum(axis=(1, 3))
        if isx == 2 and isy == 2:  # ResizeAreaFastVec (scale 2 x 2): (sum + 2) >> 2, SIMD and tail alike
            return ((s + 2) >> 2).astype(np.uint8).reshape((oh, ow) + img.shape[2:])
        out = np.clip(np.rint(s.astype(f32) * f32(1.0 / (isx * isy))), 0, 255)
        return out.astype(np.uint8).reshape((oh, ow) + img.shape[2:])
    xc, yc = _area_cells(w, ow, sx), _area_cells(h, oh, sy)
    xf = x.astype(f32)
    out = np.empty((oh, ow, x.shape[2]), np.float32)
    for dy, rows in enumerate(yc):
        acc = None
        for (r, beta) in rows:
            buf = np.zeros((ow, x.shape[2]), f32)
            for dx, cols in enumerate(xc):
                b = f32(0)
                for (c, a) in cols:
                    b = (b + xf[r, c] * a).astype(f32)
                buf[dx] = b
            t = (beta * buf).astype(f32)
            acc = t if acc is None else (acc + t).astype(f32)
        out[dy] = acc
    return np.clip(np.rint(out), 0, 255).astype(np.uint8).reshape((oh, ow) + img.shape[2:])


def area_down(gray_u8: np.ndarray, ds: int) -> np.ndarray:
    """--flow_downscale (pipeline.py:1886-1889): cv2.resize(gray, (W // ds, H // ds), INTER_AREA)."""
    h, w = gray_u8.shape
    return area_resize(gray_u8, h // ds, w // ds)


def farneback_downscaled(prev: np.ndarray, nxt: np.ndarray, ds: int) -> np.ndarray:
    """pipeline.py:1886-1892, 1920-1923: flow on the INTER_AREA-reduced grays, INTER_LINEAR back, times ds."""
    h, w = prev.shape
    small = farneback(area_down(prev, ds), area_down(nxt, ds))
    return resize_lin(small, h, w, float(ds))
