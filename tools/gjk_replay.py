"""CPU replay of the kernels' gjk_within (csrc/race_kernel.h) in float32 or float64, for the capped
queries tools/gjk_slow.py dumps: prints the per-iteration |v|, the lower bound v.w / |v| and the
simplex size, so the cause of a 48-iteration run can be read off.

usage: python tools/gjk_replay.py gpurun_out/gjk_slow_level0_2_PYB_fp32_example.npz [INDEX] [f32|f64]
"""
import sys

import numpy as np


def shape(rec, j, T):
    p = rec[17 * j:17 * j + 17].astype(T)
    return {"c": p[0:3], "R": p[3:12].reshape(3, 3), "h": p[12:15], "r": p[15], "cyl": int(rec[17 * j + 16])}


def support(s, d, T):
    dl = s["R"].T @ d
    if s["cyl"]:
        n2 = dl[0] * dl[0] + dl[1] * dl[1]
        k = s["r"] / np.sqrt(n2) if n2 > 0 else T(0)
        pl = np.array([k * dl[0], k * dl[1], s["h"][2] if dl[2] >= 0 else -s["h"][2]], T)
    else:
        pl = np.where(dl >= 0, s["h"], -s["h"]).astype(T)
    return s["c"] + s["R"] @ pl


def tri_closest(a, b, c):
    ab, ac = b - a, c - a
    d1, d2 = -ab @ a, -ac @ a
    if d1 <= 0 and d2 <= 0:
        return a, [a]
    d3, d4 = -ab @ b, -ac @ b
    if d3 >= 0 and d4 <= d3:
        return b, [b]
    vc = d1 * d4 - d3 * d2
    if vc <= 0 and d1 >= 0 and d3 <= 0:
        return a + (d1 / (d1 - d3)) * ab, [a, b]
    d5, d6 = -ab @ c, -ac @ c
    if d6 >= 0 and d5 <= d6:
        return c, [c]
    vb = d5 * d2 - d1 * d6
    if vb <= 0 and d2 >= 0 and d6 <= 0:
        return a + (d2 / (d2 - d6)) * ac, [a, c]
    va = d3 * d6 - d5 * d4
    if va <= 0 and (d4 - d3) >= 0 and (d5 - d6) >= 0:
        return b + ((d4 - d3) / ((d4 - d3) + (d5 - d6))) * (c - b), [b, c]
    den = 1 / (va + vb + vc)
    return a + (vb * den) * ab + (vc * den) * ac, [a, b, c]


def gjk_within(A0, B0, cut, T, trace=False, stall=True, v0=None, max_it=48):
    A, B = dict(A0), dict(B0)
    B["c"] = B0["c"] - A0["c"]
    A["c"] = np.zeros(3, T)
    eps, tol2 = (T(4e-6), T(1e-14)) if T == np.float32 else (T(1e-13), T(1e-26))
    W = []
    v = A["c"] - B["c"]
    if v0 is not None:
        v = np.asarray(v0, T)
    cut2 = T(cut) * T(cut)
    if v @ v < 1e-20:
        v = np.array([1, 0, 0], T)
    vv_prev = T(3e38)
    for it in range(max_it):
        w = support(A, -v, T) - support(B, v, T)
        vv, vw = v @ v, v @ w
        if stall and vv == vv_prev:
            return vv < cut2, it + 1, "stall"
        vv_prev = vv
        if trace:
            print(f"  it {it:2d} n {len(W)} |v| {np.sqrt(vv):.9g} lower {vw / np.sqrt(vv) if vv > 0 else 0:.9g}")
        if vw > 0 and vw * vw >= cut2 * vv:
            return False, it + 1, "lower"
        if vv - vw <= eps * vv:
            return vv < cut2, it + 1, "rel"
        if (vv - vw) * (vv - vw) <= tol2 * vv:
            return vv < cut2, it + 1, "abs"
        if any((q - w) @ (q - w) < 1e-20 for q in W):
            return vv < cut2, it + 1, "repeat"
        if len(W) == 0:
            W, v = [w], w
        elif len(W) == 1:
            ab = w - W[0]
            t = -(W[0] @ ab) / (ab @ ab)
            if t <= 0:
                v = W[0]
            elif t >= 1:
                W, v = [w], w
            else:
                W, v = [W[0], w], W[0] + t * ab
        elif len(W) == 2:
            v, W = tri_closest(W[0], W[1], w)
        else:
            W3 = w
            W0, W1, W2 = W
            e1, e2, e3 = W1 - W0, W2 - W0, W3 - W0
            vol = e1 @ np.cross(e2, e3)
            scl = np.sqrt((e1 @ e1) * (e2 @ e2) * (e3 @ e3))
            flat = abs(vol) <= (T(1e-5) if T == np.float32 else T(1e-12)) * scl
            best, bv, bW, outside = T(3e38), v, W, False
            faces = [(W0, W1, W2, W3), (W0, W2, W3, W1), (W0, W3, W1, W2), (W1, W3, W2, W0)]
            for p0, p1, p2, po in faces:
                nrm = np.cross(p1 - p0, p2 - p0)
                so, sd = -(nrm @ p0), nrm @ (po - p0)
                if flat or so * sd < 0:
                    outside = True
                    vf, q = tri_closest(p0, p1, p2)
                    if vf @ vf < best:
                        best, bv, bW = vf @ vf, vf, q
            if not outside:
                return True, it + 1, "inside"
            v, W = bv, bW
        if v @ v < cut2:
            return True, it + 1, "upper"
    return v @ v < cut2, max_it, "cap"


if __name__ == "__main__":
    d = np.load(sys.argv[1])
    rec = d["rec"]
    T = np.float64 if (len(sys.argv) > 3 and sys.argv[3] == "f64") else np.float32
    which = [int(sys.argv[2])] if len(sys.argv) > 2 else range(len(rec))
    for i in which:
        r = rec[i]
        A, B = shape(r, 0, T), shape(r, 1, T)
        seeded = len(r) > 42 and r[42] > 0
        res = gjk_within(A, B, r[34], T, trace=len(which) == 1, v0=r[39:42] if seeded else None,
                         max_it=int(r[43]) if len(r) > 43 else 48)
        print(i, "cut", r[34], "kinds", A["cyl"], B["cyl"], "A h/r", A["h"], A["r"], "B h/r", B["h"], B["r"],
              "|dc|", np.linalg.norm(B["c"] - A["c"]), "->", res)
