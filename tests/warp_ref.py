"""numpy restatement of cvTransformImage (src/opencv/opencv.cpp:242-309) = OpenCV
warpPerspective (imgwarp.cpp, BORDER_CONSTANT 0, no WARP_INVERSE_MAP) on the flipped image
(src/registration/registration.c:719-723).  Test infrastructure only; OpenCV itself is not
available here and its version is unpinned, so this pins the GPU kernel to the published
algorithm (float32 coefficient tables, float32 sums in OpenCV's order), not to an OpenCV
build: parity unpinned."""
import numpy as np

F = np.float32
INT_MIN, INT_MAX = -2147483648.0, 2147483647.0


def invert3(a):
    a = [float(v) for v in np.asarray(a, dtype=np.float64).reshape(9)]
    d = a[0] * (a[4] * a[8] - a[5] * a[7]) - a[1] * (a[3] * a[8] - a[5] * a[6]) + a[2] * (a[3] * a[7] - a[4] * a[6])
    if d == 0.0:
        return [0.0] * 9
    t = 1.0 / d
    return [(a[4] * a[8] - a[5] * a[7]) * t, (a[2] * a[7] - a[1] * a[8]) * t, (a[1] * a[5] - a[2] * a[4]) * t,
            (a[5] * a[6] - a[3] * a[8]) * t, (a[0] * a[8] - a[2] * a[6]) * t, (a[2] * a[3] - a[0] * a[5]) * t,
            (a[3] * a[7] - a[4] * a[6]) * t, (a[1] * a[6] - a[0] * a[7]) * t, (a[0] * a[4] - a[1] * a[3]) * t]


def coeffs(interp, x):
    x = F(x)
    if interp == 1:
        return [F(1) - x, x]
    if interp == 3:
        A = F(-0.75)
        c0 = ((A * (x + F(1)) - F(5) * A) * (x + F(1)) + F(8) * A) * (x + F(1)) - F(4) * A
        c1 = ((A + F(2)) * x - (A + F(3))) * x * x + F(1)
        c2 = ((A + F(2)) * (F(1) - x) - (A + F(3))) * (F(1) - x) * (F(1) - x) + F(1)
        c3 = F(1) - c0 - c1 - c2
        return [c0, c1, c2, c3]
    s45 = 0.70710678118654752440084436210485
    cs = [(1, 0), (-s45, -s45), (0, 1), (s45, -s45), (-1, 0), (s45, s45), (0, -1), (-s45, s45)]
    if x < F(1.192092896e-07):
        k = [F(0)] * 8
        k[3] = F(1)
        return k
    y0 = -float(x + F(3)) * np.pi * 0.25
    s0, c0 = np.sin(y0), np.cos(y0)
    k, tot = [], F(0)
    for i in range(8):
        y = -float(x + F(3) - F(i)) * np.pi * 0.25
        k.append(F((cs[i][0] * s0 + cs[i][1] * c0) / (y * y)))
        tot = F(tot + k[-1])
    tot = F(1) / tot
    return [F(v * tot) for v in k]


def table(interp):
    K = {1: 2, 3: 4, 4: 8}[interp]
    t1 = [coeffs(interp, F(i) * F(1.0 / 32)) for i in range(32)]
    tab = np.zeros((1024, K * K), dtype=np.float32)
    for i in range(32):
        for j in range(32):
            for k1 in range(K):
                for k2 in range(K):
                    tab[i * 32 + j, k1 * K + k2] = F(t1[i][k1] * t1[j][k2])
    return tab, K


def warp(img, hom, out_size=None, interp=1):
    img = np.asarray(img, dtype=np.uint16)
    C, H, W = img.shape
    oW, oH = out_size if out_size else (W, H)
    if interp == 2:
        interp = 1
    M = invert3(hom)
    bh0 = min(16, oH)
    bw = max(1, min(1024 // bh0, oW))
    yd, x = np.meshgrid(np.arange(oH, dtype=np.float64), np.arange(oW, dtype=np.float64), indexing="ij")
    xb = np.floor(x / bw) * bw
    x1 = x - xb
    X0 = M[0] * xb + M[1] * yd + M[2]
    Y0 = M[3] * xb + M[4] * yd + M[5]
    W0 = M[6] * xb + M[7] * yd + M[8]
    Wd = W0 + M[6] * x1
    disp = img[:, ::-1, :].astype(np.float32)          # display (top-down) source

    def src(c, xs, ys):
        ok = (xs >= 0) & (xs < W) & (ys >= 0) & (ys < H)
        v = np.zeros(xs.shape, dtype=np.float32)
        v[ok] = disp[c][ys[ok], xs[ok]]
        return v, ok

    out = np.zeros((C, oH, oW), dtype=np.uint16)
    with np.errstate(divide="ignore", invalid="ignore"):
        if interp == 0:
            Wi = np.where(Wd != 0, 1.0 / Wd, 0.0)
            X = np.clip(np.rint(np.clip((X0 + M[0] * x1) * Wi, INT_MIN, INT_MAX)), -32768, 32767).astype(np.int64)
            Y = np.clip(np.rint(np.clip((Y0 + M[3] * x1) * Wi, INT_MIN, INT_MAX)), -32768, 32767).astype(np.int64)
            for c in range(C):
                v, ok = src(c, X, Y)
                out[c] = v.astype(np.uint16)[::-1]
            return out
        tab, K = table(interp)
        Wi = np.where(Wd != 0, 32.0 / Wd, 0.0)
        X = np.rint(np.clip((X0 + M[0] * x1) * Wi, INT_MIN, INT_MAX)).astype(np.int64)
        Y = np.rint(np.clip((Y0 + M[3] * x1) * Wi, INT_MIN, INT_MAX)).astype(np.int64)
        sx = np.clip(X >> 5, -32768, 32767) - (K // 2 - 1)
        sy = np.clip(Y >> 5, -32768, 32767) - (K // 2 - 1)
        wt = tab[(Y & 31) * 32 + (X & 31)]              # [oH][oW][K*K]
        allout = (sx >= W) | (sx + K - 1 < 0) | (sy >= H) | (sy + K - 1 < 0)
        inside = (sx >= 0) & (sx + K <= W) & (sy >= 0) & (sy + K <= H)
        for c in range(C):
            taps = [[src(c, sx + t, sy + r) for t in range(K)] for r in range(K)]
            if K == 2:
                s = taps[0][0][0] * wt[..., 0] + taps[0][1][0] * wt[..., 1]
                s = s + taps[1][0][0] * wt[..., 2]
                s = s + taps[1][1][0] * wt[..., 3]
            else:
                si = None
                for r in range(K):
                    row = taps[r][0][0] * wt[..., r * K]
                    for t in range(1, K):
                        row = row + taps[r][t][0] * wt[..., r * K + t]
                    si = row if si is None else si + row
                sb = np.zeros(X.shape, dtype=np.float32)
                for r in range(K):
                    for t in range(K):
                        v, ok = taps[r][t]
                        sb = np.where(ok, sb + v * wt[..., r * K + t], sb).astype(np.float32)
                s = np.where(inside, si, sb)
            r = np.rint(s.astype(np.float32))
            v = np.clip(r, 0, 65535).astype(np.uint16)
            v[allout] = 0
            out[c] = v[::-1]
    return out
