"""Independent float64 NumPy restatement of the SiftGPU hot path (test infrastructure).

Purpose: cross-check the C++ oracle (oracle/sift_oracle.cpp) with code that shares none of its
structure or arithmetic: float64 throughout, libm/NumPy transcendentals instead of
sift_math.h, vectorised filters, a plain 26-neighbour extremum test instead of the
ComputeKEY state machine, np.add.at histograms instead of ordered fma chains.  Agreement within
float32 rounding (tests/test_ref_numpy.py) shows that the oracle restates the reference's
algorithm rather than merely agreeing with the HIP kernels.  Reference lines followed:

  sigma schedule / taps   SiftGPU.cpp:446-498, ProgramCU.cu:375-403
  filter + downsample     ProgramCU.cu:115-222 (clamp-to-edge separable), :287-298
  DoG + key test          ProgramCU.cu:485-531, 553-694 (contrast, extremum, edge, 3x3 solve)
  orientation             ProgramCU.cu:813-977 (square window; circular per ProgramCU-0.cu:834)
  descriptor + normalise  ProgramCU.cu:1013-1101, 1173-1208
"""
import math

import numpy as np


def schedule(d=3, filter_factor=4.0, dog_threshold=0.0, edge_threshold=0.0, octave_min=0):
    """SiftParam::ParseSiftParam / GetInitialSmoothSigma (SiftGPU.cpp:446-498): the first
    level's smoothing assumes the input already carries sigma_n = 0.5 at octave 0, i.e.
    0.5 / 2^octave_min in the first octave's pixels."""
    sigma0 = 1.6 * 2.0 ** (1.0 / d)
    sigmak = 2.0 ** (1.0 / d)
    dsigma0 = sigma0 * math.sqrt(1.0 - 1.0 / (sigmak * sigmak))
    level_min, level_max = -1, d + 1
    sig = [dsigma0 * sigmak ** i for i in range(level_min + 1, level_max + 1)]
    a = sigma0 * 2.0 ** (level_min / d)
    b = 0.5 / 2.0 ** octave_min
    initial = math.sqrt(a * a - b * b) if a > b + 0.001 else 0.0
    return {
        "d": d, "nlev": d + 3, "sigma0": sigma0, "level_sigma": [sigma0 * 2.0 ** ((j + 1) / d) for j in range(d)],
        "filter_sigma": sig, "initial": initial, "factor": filter_factor,
        "t": dog_threshold if dog_threshold > 0 else 0.02 / d,
        "edge": edge_threshold if edge_threshold > 0 else 10.0,
    }


def taps(sigma, factor):
    sz = int(math.ceil(factor * sigma - 0.5))
    width = 2 * sz + 1
    if width > 33:
        sz = 16
    elif width < 5:
        sz = 2
    i = np.arange(-sz, sz + 1, dtype=np.float64)
    k = np.exp(-0.5 * i * i / (sigma * sigma))
    return k / k.sum()


def gfilter(img, k):
    half = len(k) // 2
    h, w = img.shape
    p = np.pad(img, ((0, 0), (half, half)), mode="edge")
    t = sum(k[i] * p[:, i:i + w] for i in range(len(k)))
    p = np.pad(t, ((half, half), (0, 0)), mode="edge")
    return sum(k[i] * p[i:i + h, :] for i in range(len(k)))


def geometry(w, h, octave_num):
    w &= ~3
    n = octave_num if octave_num >= 1 else max(1, int(math.floor(math.log2(min(w, h)))) - 3)
    out = []
    for _ in range(n):
        out.append((w, h, (w + 3) // 4 * 4))
        w >>= 1
        h >>= 1
    return out


def upsample(img, s):
    """UpsampleKernel<s> (ProgramCU.cu:225-269) in float64: the image bound as one flat buffer,
    so the right neighbour of a row's last pixel is the next row's first one and reads past
    the buffer are 0; output row R blends source rows R >> s and (R >> s) + 1 with weight
    (R & (S-1)) / S, and source column c fills the S outputs c S .. c S + S-1 between pixels c
    and c + 1."""
    S = 1 << s
    h, w = img.shape
    flat = np.concatenate([img.reshape(-1), np.zeros(w + 2)])
    out = np.zeros((h * S, w * S))
    cols = np.arange(w)
    for R in range(h * S):
        r, f = R >> s, (R & (S - 1)) / S
        i = r * w + cols
        v1 = (1 - f) * flat[i] + f * flat[i + w]
        v2 = (1 - f) * flat[i + 1] + f * flat[i + w + 1]
        for k in range(S):
            out[R, cols * S + k] = v1 * (1 - k / S) + v2 * (k / S)
    return out


def pyramid(img_u8, S, octave_num=-1, octave_min=0):
    """[octave][level] float64 Gaussian images, each wa x h.  octave_min < 0 (-fo): the input
    (width truncated to a multiple of 4) upsampled by 2^-octave_min first (PyramidCU.cpp:89-112,
    SampleImageU)."""
    h, w = img_u8.shape
    base = img_u8[:, : w & ~3].astype(np.float64) / 255.0
    if octave_min < 0:
        base = upsample(base, -octave_min)
    geo = geometry(base.shape[1], base.shape[0], octave_num)
    base = base[:, : geo[0][2]]
    out = []
    for o, (_, ho, wa) in enumerate(geo):
        if o == 0:
            g0 = gfilter(base, taps(S["initial"], S["factor"]))
        else:
            src = out[-1][S["d"]]   # level_ds - level_min = d (PyramidCU.cpp:1024)
            cols = np.minimum(2 * np.arange(wa), src.shape[1] - 1)
            g0 = src[0:2 * ho:2, :][:, cols]
        lv = [g0]
        for k in range(1, S["nlev"]):
            lv.append(gfilter(lv[-1], taps(S["filter_sigma"][k - 1], S["factor"])))
        out.append(lv)
    return out


def _solve3(A, b):
    """Gaussian elimination with partial pivoting; None when a pivot is below 1e-10 (the
    reference then keeps the integer position, ProgramCU.cu:631-667)."""
    M = np.concatenate([A, b[:, None]], axis=1).astype(np.float64)
    for c in range(3):
        r = c + int(np.argmax(np.abs(M[c:, c])))
        if abs(M[r, c]) < 1e-10:
            return None
        M[[c, r]] = M[[r, c]]
        M[c] /= M[c, c]
        for rr in range(c + 1, 3):
            M[rr] -= M[rr, c] * M[c]
    x = np.zeros(3)
    for c in (2, 1, 0):
        x[c] = M[c, 3] - M[c, c + 1:3] @ x[c + 1:3]
    return x


def detect(G, S, subpixel=True):
    """Candidates per (octave, j): list of (col, row, dx, dy, ds, sign) in raster order."""
    t0 = (0.8 if subpixel else 1.0) * S["t"]
    res = {}
    for o, lv in enumerate(G):
        D = [lv[m] - lv[m - 1] for m in range(1, S["nlev"])]
        h, w = D[0].shape
        for j in range(S["d"]):
            P, C, N = D[j], D[j + 1], D[j + 2]
            v = C[1:-1, 1:-1]
            nb = []
            for plane in (P, C, N):
                for dy in (-1, 0, 1):
                    for dx in (-1, 0, 1):
                        if plane is C and dy == 0 and dx == 0:
                            continue
                        nb.append(plane[1 + dy:h - 1 + dy, 1 + dx:w - 1 + dx])
            nb = np.stack(nb)
            ext = (np.abs(v) > t0) & ((v > nb.max(0)) | (v < nb.min(0)))
            rows, cols = np.nonzero(ext)
            out = []
            for r, c in zip(rows + 1, cols + 1):
                vv = C[r, c]
                fxx = C[r, c - 1] + C[r, c + 1] - 2 * vv
                fyy = C[r - 1, c] + C[r + 1, c] - 2 * vv
                fxy = 0.25 * (C[r + 1, c + 1] + C[r - 1, c - 1] - C[r + 1, c - 1] - C[r - 1, c + 1])
                det = fxx * fyy - fxy * fxy
                tr = fxx + fyy
                if det <= 0 or tr * tr > (S["edge"] + 1) ** 2 / S["edge"] * det:
                    continue
                dx = dy = ds = 0.0
                if subpixel:
                    fx = 0.5 * (C[r, c + 1] - C[r, c - 1])
                    fy = 0.5 * (C[r + 1, c] - C[r - 1, c])
                    fs = 0.5 * (N[r, c] - P[r, c])
                    fss = N[r, c] + P[r, c] - 2 * vv
                    fxs = 0.25 * (N[r, c + 1] + P[r, c - 1] - N[r, c - 1] - P[r, c + 1])
                    fys = 0.25 * (N[r + 1, c] + P[r - 1, c] - N[r - 1, c] - P[r + 1, c])
                    A = np.array([[fxx, fxy, fxs], [fxy, fyy, fys], [fxs, fys, fss]])
                    x = _solve3(A, -np.array([fx, fy, fs]))
                    if x is not None:
                        dx, dy, ds = x
                        if not (abs(vv + 0.5 * (dx * fx + dy * fy + ds * fs)) > S["t"]
                                and max(abs(dx), abs(dy), abs(ds)) < 1.0):
                            continue
                out.append((c, r, dx, dy, ds, 1.0 if vv > 0 else -1.0))
            res[(o, j)] = out
    return res


def gradient(g):
    gy, gx = np.zeros_like(g), np.zeros_like(g)
    gx[:, 1:-1] = g[:, 2:] - g[:, :-2]
    gy[1:-1, :] = g[2:, :] - g[:-2, :]
    return 0.5 * np.hypot(gx, gy), np.arctan2(gy, gx)


def orientation(mag, ang, x, y, s, circular=False, max_orientation=2):
    """Orientation angles (radians, the reference's internal convention) of a keypoint at
    octave coordinates (x, y) and scale s."""
    H, W = mag.shape
    win = abs(s) * 3.0
    gs = s * 1.5
    xmin = max(1.5, math.floor(x - win) + 0.5)
    ymin = max(1.5, math.floor(y - win) + 0.5)
    xmax = min(W - 1.5, math.floor(x + win) + 0.5)
    ymax = min(H - 1.5, math.floor(y + win) + 0.5)
    xs = np.arange(xmin, xmax + 0.5)
    ys = np.arange(ymin, ymax + 0.5)
    X, Y = np.meshgrid(xs, ys)
    sq = (X - x) ** 2 + (Y - y) ** 2
    keep = np.ones_like(sq, bool) if not circular else sq < win * win + 0.5
    xi, yi = X.astype(int)[keep], Y.astype(int)[keep]
    wgt = mag[yi, xi] * np.exp(-sq[keep] / (2 * gs * gs))
    b = np.floor(ang[yi, xi] * 36 / (2 * math.pi)).astype(int) % 36
    hist = np.zeros(36)
    np.add.at(hist, b, wgt)
    for _ in range(6):
        hist = (np.roll(hist, 1) + hist + np.roll(hist, -1)) / 3.0
    if max_orientation == 1:
        i = int(np.argmax(hist))
        p, n = hist[i - 1], hist[(i + 1) % 36]
        return [(i + 0.5 + 0.5 * (n - p) / (2 * hist[i] - n - p)) * 2 * math.pi / 36]
    thr = 0.8 * hist.max()
    peaks = []
    for i in range(36):
        p, n = hist[i - 1], hist[(i + 1) % 36]
        if hist[i] > thr and hist[i] > p and hist[i] > n:
            peaks.append((hist[i], i + 0.5 + 0.5 * (n - p) / (2 * hist[i] - n - p)))
    peaks.sort(key=lambda t: -t[0])
    return [r * 2 * math.pi / 36 for _, r in peaks[:2]]


def descriptor(mag, ang, x, y, s, o, window_factor=3.0, normalize=True):
    H, W = mag.shape
    spt = abs(s * window_factor)
    c, sn = math.cos(o), math.sin(o)
    anglef = o - 2 * math.pi if o > math.pi else o
    des = np.zeros((16, 9))
    for bidx in range(16):
        ix, iy = bidx & 3, bidx >> 2
        ox, oy = ix - 1.5, iy - 1.5
        ptx = c * spt * ox - sn * spt * oy + x
        pty = c * spt * oy + sn * spt * ox + y
        bsz = abs(c * spt) + abs(sn * spt)
        xmin = max(1.5, math.floor(ptx - bsz) + 0.5)
        ymin = max(1.5, math.floor(pty - bsz) + 0.5)
        xmax = min(W - 1.5, math.floor(ptx + bsz) + 0.5)
        ymax = min(H - 1.5, math.floor(pty + bsz) + 0.5)
        if xmax < xmin or ymax < ymin:
            continue
        X, Y = np.meshgrid(np.arange(xmin, xmax + 0.5), np.arange(ymin, ymax + 0.5))
        dx, dy = X - ptx, Y - pty
        nx = (c * dx + sn * dy) / spt
        ny = (c * dy - sn * dx) / spt
        keep = (np.abs(nx) < 1) & (np.abs(ny) < 1)
        nx, ny = nx[keep], ny[keep]
        xi, yi = X.astype(int)[keep], Y.astype(int)[keep]
        w = (np.exp(-0.125 * ((nx + ox) ** 2 + (ny + oy) ** 2)) * (1 - np.abs(nx)) *
             (1 - np.abs(ny)) * mag[yi, xi])
        theta = (anglef - ang[yi, xi]) * 4 / math.pi
        theta = np.where(theta < 0, theta + 8, theta)
        f = np.floor(theta).astype(int)
        ok = f < 8
        np.add.at(des[bidx], f[ok], ((f + 1 - theta) * w)[ok])
        np.add.at(des[bidx], f[ok] + 1, ((theta - f) * w)[ok])
    des[:, 0] += des[:, 8]
    d = des[:, :8].reshape(128)
    if normalize:
        d = d / np.sqrt((d * d).sum())
        d = np.minimum(d, 0.2)
        d = d / np.sqrt((d * d).sum())
    return d
