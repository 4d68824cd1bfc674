"""Numerics of a Winograd F(2x2, 3x3) bf16x3 res block conv, against the
direct bf16x3 conv the kernels run, on the res golden fixtures.

Within each (row-class, column-class) sub-grid a dilated 3x3 conv is a plain 3x3 conv
(model.py:94-98), so F(2x2,3x3) applies per class: input tiles d (4x4, stride 2),
V = B^T d B (fp32), U = G g G^T (fp32, factors of 1/2), M = sum_c U V over channels,
Y = A^T M A (fp32).  bf16x3: V and U each split into bf16 (hi, lo); products
Uh Vh + Uh Vl + Ul Vh, accumulated in fp32 (float64 sum of the exact products, rounded
to fp32 per 32-deep MFMA k-step chunk -- the matrix core's fp32 accumulation).
Layer inputs are the fp32 post-BN maps; everything else (ReLU, residual, BN, mean,
Linear) is float64 as in oracle/ref_numpy.py.  Prints the max logit error vs the
float64 oracle for (a) the direct bf16x3 conv and (b) Winograd bf16x3.

    python exp/winograd_sim.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
from oracle import ref_numpy as orc  # noqa: E402
from golden_util import fixture_names, load_fixture  # noqa: E402

BT = np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], np.float32)
G = np.array([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]], np.float32)
AT = np.array([[1, 1, 1, 0], [0, 1, -1, -1]], np.float32)


def bf16(x):
    u = np.ascontiguousarray(np.asarray(x, np.float32)).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return u.view(np.float32)


def split(x):
    x = np.asarray(x, np.float32)
    h = bf16(x)
    return h, bf16(x - h)


def mm_x3(uh, ul, vh, vl, kchunk=32):
    """sum_c U[o, c] V[c, t] as hi*hi + hi*lo + lo*hi, fp32 accumulation per 32-deep chunk."""
    acc = np.zeros((uh.shape[0], vh.shape[1]), np.float32)
    for c0 in range(0, uh.shape[1], kchunk):
        s = slice(c0, c0 + kchunk)
        part = (uh[:, s].astype(np.float64) @ vh[s].astype(np.float64) + uh[:, s].astype(np.float64) @ vl[s]
                + ul[:, s].astype(np.float64) @ vh[s])
        acc = (acc.astype(np.float64) + part).astype(np.float32)
    return acc


def conv_direct_x3(x, w, d):
    """The direct bf16x3 dilated conv (the kernels' arithmetic, K = 9 C)."""
    x = np.asarray(x, np.float32)
    n, c, h, wd = x.shape
    xp = np.pad(x, ((0, 0), (0, 0), (d, d), (d, d)))
    win = np.lib.stride_tricks.sliding_window_view(xp, (2 * d + 1, 2 * d + 1), axis=(2, 3))[..., ::d, ::d]
    cols = win.transpose(1, 4, 5, 0, 2, 3).reshape(c * 9, -1)           # (c, ky, kx) x (n, h, w)
    wh, wl = split(np.asarray(w, np.float32).reshape(w.shape[0], -1))
    xh, xl = split(cols)
    y = mm_x3(wh, wl, xh, xl)
    return y.reshape(w.shape[0], n, h, wd).transpose(1, 0, 2, 3).astype(np.float64)


def conv_winograd_x3(x, w, d):
    x = np.asarray(x, np.float32)
    n, c, h, wd = x.shape
    o = w.shape[0]
    U = np.einsum("aj,ocjk,bk->aboc", G, np.asarray(w, np.float32), G).astype(np.float32)  # 4 4 o c
    uh, ul = split(U)
    out = np.zeros((n, o, h, wd), np.float64)
    for r in range(d):
        for s in range(d):
            xc = x[:, :, r::d, s::d]
            hc, wc = xc.shape[2], xc.shape[3]
            th, tw = (hc + 1) // 2, (wc + 1) // 2
            xp = np.zeros((n, c, 2 * th + 2, 2 * tw + 2), np.float32)
            xp[:, :, 1:1 + hc, 1:1 + wc] = xc
            tiles = np.lib.stride_tricks.sliding_window_view(xp, (4, 4), axis=(2, 3))[:, :, ::2, ::2]  # n c th tw 4 4
            V = np.einsum("ij,nctvjk,lk->ilcntv", BT, tiles, BT).astype(np.float32)  # 4 4 c n th tw
            vh, vl = split(V.reshape(4, 4, c, -1))
            M = np.empty((4, 4, o, vh.shape[-1]), np.float32)
            for a in range(4):
                for b in range(4):
                    M[a, b] = mm_x3(uh[a, b], ul[a, b], vh[a, b], vl[a, b])
            Y = np.einsum("ij,jkot,lk->ilot", AT, M, AT).astype(np.float32)                 # 2 2 o (n th tw)
            Y = Y.reshape(2, 2, o, n, th, tw).transpose(3, 2, 4, 0, 5, 1).reshape(n, o, 2 * th, 2 * tw)
            out[:, :, r::d, s::d] = Y[:, :, :hc, :wc]
    return out


def res_forward(params, cfg, x, conv):
    x = np.asarray(x, np.float64)[:, None]
    old = None
    for i in range(int(cfg["n_layers"]) + 1):
        if i == 0:
            y = orc.relu(orc.conv2d(x, params["conv0.weight"], padding=(1, 1)))
            if "res_pool" in cfg:
                y = orc.avg_pool2d(y, tuple(cfg["res_pool"]))
            old = x = y
            continue
        dd = orc.res_dilation(cfg, i)
        y = orc.relu(conv(x, params[f"conv{i}.weight"], dd))
        if i % 2 == 0:
            x = old = y + old
        else:
            x = y
        x = orc.batch_norm_eval(x, params[f"bn{i}.running_mean"], params[f"bn{i}.running_var"])
    z = x.reshape(x.shape[0], x.shape[1], -1).mean(axis=2)
    return orc.linear(z, params["output.weight"], params["output.bias"])


def main():
    worst = {"direct": 0.0, "winograd": 0.0}
    for name in fixture_names():
        if not name.startswith("res"):
            continue
        cfg, params, x, logits, meta = load_fixture(name)
        ref = orc.forward(params, cfg, x)
        e_d = float(np.abs(res_forward(params, cfg, x, conv_direct_x3) - ref).max())
        e_w = float(np.abs(res_forward(params, cfg, x, conv_winograd_x3) - ref).max())
        worst["direct"] = max(worst["direct"], e_d)
        worst["winograd"] = max(worst["winograd"], e_w)
        print(f"{name:22s} max |logit err| vs float64: direct bf16x3 {e_d:.2e}   Winograd bf16x3 {e_w:.2e}", flush=True)
    print("worst:", worst)


if __name__ == "__main__":
    main()
