"""Independent numpy / pure-Python restatement of the reference stackers (TEST INFRASTRUCTURE
ONLY).  Used to cross-check the C oracle (oracle/*.c) on small inputs; neither is ever on
the product path.  Written from the reference sources, not from the C oracle:

  GSL mean / sd   third-party (GSL statistics/mean_source.c, variance_source.c): running
                  recurrences in long double (numpy.longdouble = x87 80-bit on x86-64)
  median_sorted   gsl_stats_ushort_median_from_sorted_data
  round_to_WORD   src/core/utils.c:68-74
  rejection loop  src/stacking/stacking.c:1656-1794 (+ helpers :1130-1187)
  stack_median    src/stacking/stacking.c:746-769
  stack_summing   src/stacking/stacking.c:297-342
  quality         src/algos/quality.c:46-349
"""
import math

import numpy as np

LD = np.longdouble


def round_to_word(x):
    if x != x:
        # (WORD)(NaN + 0.5): x86-64 cvttsd2si yields 0x80000000, truncated to 0 (the
        # reference reaches this when stale rejected[] entries empty the stack)
        return 0
    if x <= 0.0:
        return 0
    if x > 65535.0:
        return 65535
    return int(x + 0.5)


def gsl_mean(data):
    mean = LD(0)
    for i, v in enumerate(data):
        mean += (LD(int(v)) - mean) / LD(i + 1)
    return float(mean)


def gsl_sd(data):
    n = len(data)
    mean = gsl_mean(data)                   # rounded to double
    var = LD(0)
    for i, v in enumerate(data):
        delta = LD(float(int(v)) - mean)    # ushort - double in double, then widened
        var += (delta * delta - var) / LD(i + 1)
    var = float(var)
    return math.sqrt(var * (float(n) / float(n - 1)))


def median_sorted(s):
    n = len(s)
    if n == 0:
        return 0.0
    lhs, rhs = (n - 1) // 2, n // 2
    if lhs == rhs:
        return float(s[lhs])
    return (int(s[lhs]) + int(s[rhs])) / 2.0


def fit_linear(x, y):
    m_x = m_y = m_dx2 = m_dxdy = 0.0
    for i in range(len(x)):
        m_x += (x[i] - m_x) / (i + 1.0)
        m_y += (y[i] - m_y) / (i + 1.0)
    for i in range(len(x)):
        dx = x[i] - m_x
        dy = y[i] - m_y
        m_dx2 += (dx * dx - m_dx2) / (i + 1.0)
        m_dxdy += (dx * dy - m_dxdy) / (i + 1.0)
    b = fdiv(m_dxdy, m_dx2)
    return m_y - m_x * b, b


def fdiv(a, b):
    """IEEE double division (C semantics: x/0 = +-inf, 0/0 = nan)."""
    if b == 0.0:
        if a == 0.0 or a != a:
            return float("nan")
        return math.copysign(float("inf"), a) * math.copysign(1.0, b)
    return a / b


def _clip(px, sl, sh, sigma, median, crej):
    if median - px > sl * sigma:
        crej[0] += 1
        return -1
    if px - median > sh * sigma:
        crej[1] += 1
        return 1
    return 0


def reject_pixel(stack, rejected, rejection, sig, crej):
    """One pixel of stacking.c:1656-1794.  `stack` is the gathered column (frame order),
    `rejected` the thread's carried rejected[] array (mutated, as in the reference)."""
    stack = [int(v) for v in stack]
    N = len(stack)
    sl, sh = sig
    r = 0
    if rejection == 1:            # PERCENTILE
        stack.sort()
        median = median_sorted(stack)
        for f in range(N):
            v = 0
            if fdiv(median - stack[f], median) > sl:
                crej[0] += 1
                v = -1
            elif fdiv(stack[f] - median, median) > sh:
                crej[1] += 1
                v = 1
            rejected[f] = v
        frame, j = 0, 0
        while frame < N:
            if rejected[j] != 0 and N > 1:
                del stack[frame]
                frame -= 1
                N -= 1
            frame += 1
            j += 1
    elif rejection in (2, 4, 5):  # SIGMA, WINSORIZED, LINEARFIT
        while True:
            if rejection == 5:
                stack[:N] = sorted(stack[:N])
                a0, a1 = fit_linear([float(i) for i in range(N)], [float(v) for v in stack[:N]])
                b, a = a0, a1
                sigma = 0.0
                for f in range(N):
                    sigma += abs(stack[f] - (a * f + b))
                sigma /= N
            else:
                sigma = gsl_sd(stack[:N])
                stack[:N] = sorted(stack[:N])
                median = median_sorted(stack[:N])
            if rejection == 4:
                w = list(stack[:N])
                while True:
                    m0 = median - 1.5 * sigma
                    m1 = median + 1.5 * sigma
                    for jj in range(N):
                        if w[jj] < m0:
                            w[jj] = round_to_word(m0)
                        elif w[jj] > m1:
                            w[jj] = round_to_word(m1)
                    w.sort()
                    median = median_sorted(w)
                    sigma0 = sigma
                    sigma = 1.134 * gsl_sd(w)
                    q = fdiv(abs(sigma - sigma0), sigma0)
                    if not (q > 0.0005):
                        break
            n = 0
            frame = 0
            while frame < N:
                if rejection == 5:
                    v = 0
                    if fdiv(a * frame + b - stack[frame], sigma) > sl:
                        crej[0] += 1
                        v = -1
                    elif fdiv(stack[frame] - a * frame - b, sigma) > sh:
                        crej[1] += 1
                        v = 1
                    rejected[frame] = v
                else:
                    rejected[frame] = _clip(stack[frame], sl, sh, sigma, median, crej)
                if rejected[frame]:
                    r += 1
                if N - r <= 4:
                    break
                frame += 1
            frame, j = 0, 0
            while frame < N - n:
                if rejected[j] != 0:
                    del stack[frame]
                    stack.append(0)
                    n += 1
                    frame -= 1
                frame += 1
                j += 1
            N -= n
            if not (n > 0 and N > 3):
                break
    elif rejection == 3:          # SIGMEDIAN
        while True:
            sigma = gsl_sd(stack[:N])
            stack[:N] = sorted(stack[:N])
            median = median_sorted(stack[:N])
            n = 0
            for f in range(N):
                if _clip(stack[f], sl, sh, sigma, median, crej):
                    stack[f] = round_to_word(median)
                    n += 1
            if not (n > 0 and N > 3):
                break
    s = 0.0
    for f in range(N):
        s += stack[f]
    return round_to_word(fdiv(s, float(N)))


def stack_rejection_1thread(frames, rejection, sig, shiftx=None, shifty=None, rows=None):
    """stack_mean_with_rejection with one OpenMP thread and one block per channel-quarter
    order (blocks top-down, channel-major); frames [N][C][H][W] memory order (bottom-up).
    rows = (begin, end): only memory rows [begin, end) (a row band) are written and counted,
    others stay 0.  Every pixel the thread visits before the band is still stacked, so the
    stale rejected[] a band pixel inherits (SURVEY a3 iii) is the full run's."""
    N, C, H, W = frames.shape
    out = np.zeros((C, H, W), dtype=np.uint16)
    rej = np.zeros((3, 2), dtype=np.uint64)
    rejected = [0] * N
    last = None                         # (c, t) of the band's last pixel row in thread order
    if rows is not None:
        last = (C - 1, H - rows[0])
    for c in range(C):
        for t in range(H):              # top-down rows, as the block loop visits them
            R = H - 1 - t
            if last is not None and (c, t) >= last:
                break
            crej = [0, 0]
            for x in range(W):
                col = []
                for f in range(N):
                    sx = int(shiftx[f]) if shiftx is not None else 0
                    sy = int(shifty[f]) if shifty is not None else 0
                    if sx and not (0 <= x - sx < W):
                        col.append(0)
                        continue
                    sr = R - sy
                    col.append(int(frames[f, c, sr, x - sx]) if 0 <= sr < H else 0)
                out[c, R, x] = reject_pixel(col, rejected, rejection, sig, crej)
            if rows is not None and not (rows[0] <= R < rows[1]):
                out[c, R] = 0           # before the band: stacked for its state only
                continue
            rej[c, 0] += crej[0]
            rej[c, 1] += crej[1]
    return out, rej


def stack_median(frames):
    N, C, H, W = frames.shape
    s = np.sort(frames.astype(np.int64), axis=0)
    lhs, rhs = (N - 1) // 2, N // 2
    med = (s[lhs] + s[rhs]) / 2.0
    return np.floor(med).astype(np.uint16)   # implicit double -> WORD truncation


def stack_summing(frames, shiftx=None, shifty=None):
    N, C, H, W = frames.shape
    acc = np.zeros((C, H, W), dtype=np.uint64)
    for f in range(N):
        sx = int(shiftx[f]) if shiftx is not None else 0
        sy = int(shifty[f]) if shifty is not None else 0
        src = np.zeros((C, H, W), dtype=np.uint64)
        ys, xs = np.mgrid[0:H, 0:W]
        ny, nx = ys - sy, xs - sx
        ok = (nx >= 0) & (nx < W) & (ny >= 0) & (ny < H)
        ok &= (ny * W + nx) > 0                 # `ii > 0`: source pixel 0 never summed
        src[:, ok] = frames[f][:, ny[ok], nx[ok]]
        acc += src
    maxim = int(acc.max())
    out = np.zeros((C, H, W), dtype=np.uint16)
    ratio = 65535.0 / maxim if maxim > 65535 else 1.0
    flat = acc.reshape(-1)
    o = out.reshape(-1)
    for k in range(flat.size):
        o[k] = round_to_word(float(flat[k]) if ratio == 1.0 else float(flat[k]) * ratio)
    return out, maxim


def quality(img):
    """QualityEstimate, src/algos/quality.c:46-218 (see SURVEY a14 for the maxp quirk)."""
    img = np.asarray(img, dtype=np.int64)
    height, width = img.shape
    region_w, region_h = width - 1, height - 1
    dval = 0.0
    subsample = 3
    while subsample <= 5:
        xs, ys = region_w // subsample, region_h // subsample
        if xs < 2 or ys < 2:
            break
        samp = np.zeros((ys, xs), dtype=np.int64)
        for j in range(ys):
            for i in range(xs):
                blk = img[j * subsample:(j + 1) * subsample, i * subsample:(i + 1) * subsample]
                samp[j, i] = int(blk.sum()) // (subsample * subsample)
        mid = samp[1:ys - 1].reshape(-1)
        mid = mid[(mid > 0) & (mid < 65530)]
        mx = int(mid.max()) if mid.size else 0
        if mx > 0:
            mult = 60000.0 / float(mx)
            samp = np.array([[min(65535, int(float(v) * mult)) for v in row] for row in samp], dtype=np.int64)
        sm = np.zeros_like(samp)
        for y in range(1, ys - 1):
            for x in range(1, xs - 1):
                sm[y, x] = int(samp[y - 1:y + 2, x - 1:x + 2].sum()) // 9
        yb = int(ys * 0.1) + 1
        xb = int(xs * 0.1) + 1
        mp = np.zeros((ys, xs), dtype=bool)
        cnt = 0
        for y in range(yb, ys - yb):
            for x in range(xb, xs - xb):
                if sm[y, x] >= 10240:
                    mp[y - 1:y + 2, x - 1:x + 2] = True
                    cnt += 1
        if cnt == 0:
            q = -1.0
        else:
            val = 0
            pix = 0
            for y in range(yb, ys - yb):
                for x in range(xb, xs - xb):
                    if mp[y, x]:
                        d1 = int(sm[y, x]) - int(sm[y, x + 1])
                        d2 = int(sm[y, x]) - int(sm[y + 1, x])
                        val += d1 * d1 + d2 * d2
                        pix += 1
            q = float(val) / float(pix) / 10
        dval += q * ((3 * 3) // (subsample * subsample))
        subsample += 1
        while width // subsample == xs and height // subsample == ys:
            subsample += 1
    return math.sqrt(dval) if dval >= 0 else float("nan")
