"""Oracle: a plain-numpy CPU restatement of Honk's KWS forward paths.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (``honk_amd``) imports this
module; only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg
of ``bench.py`` use it, and only as the checker / the timed CPU baseline.

It restates, without torch, the two model families of the reference:

* ``SpeechResModel``  -- /root/reference/utils/model.py:82-121
* ``SpeechModel``     -- /root/reference/utils/model.py:123-205

Parity is pinned by ``tests/golden/*.npz``, produced by importing the reference
itself in the build container (``tests/golden/make_golden.py``); see
``tests/test_oracle_golden.py``.

Arithmetic: every contraction is an explicit im2col + matmul, in ``acc_dtype``
(float64 for the parity oracle, float32 for the CPU throughput baseline).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np


# --------------------------------------------------------------------------- #
# shapes: restates the constructors (model.py:82-102, 123-184)
# --------------------------------------------------------------------------- #
def res_param_shapes(cfg):
    """Ordered state_dict schema of SpeechResModel (model.py:86-102).

    Registration order: conv0, then per layer i=1..n: bn{i} then conv{i}
    (model.py:99-101), then output.
    """
    c = int(cfg["n_feature_maps"])
    n = int(cfg["n_layers"])
    shapes = OrderedDict()
    shapes["conv0.weight"] = (c, 1, 3, 3)
    for i in range(1, n + 1):
        shapes[f"bn{i}.running_mean"] = (c,)
        shapes[f"bn{i}.running_var"] = (c,)
        shapes[f"bn{i}.num_batches_tracked"] = ()
        shapes[f"conv{i}.weight"] = (c, c, 3, 3)
    shapes["output.weight"] = (int(cfg["n_labels"]), c)
    shapes["output.bias"] = (int(cfg["n_labels"]),)
    return shapes


def res_dilation(cfg, i):
    """Dilation (== padding) of conv{i}, i>=1 (model.py:93-98): convs[i-1] uses 2**((i-1)//3)."""
    if cfg.get("use_dilation"):
        return int(2 ** ((i - 1) // 3))
    return 1


def _conv_out(n, k, s):
    return (n - k) // s + 1


def cnn_geometry(cfg):
    """Shape probe of SpeechModel.__init__ (model.py:143-160), without running a net."""
    h, w = int(cfg["height"]), int(cfg["width"])
    c1 = int(cfg["n_feature_maps1"])
    k1 = tuple(cfg["conv1_size"])
    s1 = tuple(cfg["conv1_stride"])
    p1 = tuple(cfg["conv1_pool"])
    oh, ow = _conv_out(h, k1[0], s1[0]), _conv_out(w, k1[1], s1[1])
    ph, pw = oh // p1[0], ow // p1[1]
    geo = dict(conv1=(c1, oh, ow), pool1=(c1, ph, pw))
    size = c1 * ph * pw
    if "conv2_size" in cfg:
        c2 = int(cfg["n_feature_maps2"])
        k2 = tuple(cfg["conv2_size"])
        s2 = tuple(cfg["conv2_stride"])
        p2 = tuple(cfg["conv2_pool"])
        oh2, ow2 = _conv_out(ph, k2[0], s2[0]), _conv_out(pw, k2[1], s2[1])
        geo["conv2"] = (c2, oh2, ow2)
        geo["pool2"] = (c2, oh2 // p2[0], ow2 // p2[1])
        size = c2 * (oh2 // p2[0]) * (ow2 // p2[1])
    geo["flat"] = size
    return geo


def cnn_param_shapes(cfg):
    """Ordered state_dict schema of SpeechModel (model.py:135-184)."""
    geo = cnn_geometry(cfg)
    tf = bool(cfg.get("tf_variant"))
    shapes = OrderedDict()
    c1 = int(cfg["n_feature_maps1"])
    k1 = tuple(cfg["conv1_size"])
    shapes["conv1.weight"] = (c1, 1, k1[0], k1[1])
    shapes["conv1.bias"] = (c1,)
    if "conv2_size" in cfg:
        c2 = int(cfg["n_feature_maps2"])
        k2 = tuple(cfg["conv2_size"])
        shapes["conv2.weight"] = (c2, c1, k2[0], k2[1])
        shapes["conv2.bias"] = (c2,)
    last = geo["flat"]
    if not tf:
        shapes["lin.weight"] = (32, geo["flat"])
        shapes["lin.bias"] = (32,)
    if "dnn1_size" in cfg:
        d1 = int(cfg["dnn1_size"])
        shapes["dnn1.weight"] = (d1, geo["flat"] if tf else 32)
        shapes["dnn1.bias"] = (d1,)
        last = d1
        if "dnn2_size" in cfg:
            d2 = int(cfg["dnn2_size"])
            shapes["dnn2.weight"] = (d2, d1)
            shapes["dnn2.bias"] = (d2,)
            last = d2
    shapes["output.weight"] = (int(cfg["n_labels"]), last)
    shapes["output.bias"] = (int(cfg["n_labels"]),)
    return shapes


def param_shapes(name_or_cfg, cfg=None):
    cfg = cfg if cfg is not None else name_or_cfg
    if "n_layers" in cfg:
        return res_param_shapes(cfg)
    return cnn_param_shapes(cfg)


# --------------------------------------------------------------------------- #
# deterministic synthetic parameters (numpy PCG64; portable)
# --------------------------------------------------------------------------- #
def make_params(cfg, seed):
    """Kaiming-uniform-like weights U(-1/sqrt(fan_in), 1/sqrt(fan_in)) from PCG64(seed).

    BN running stats: mean ~ N(0, 0.1^2), var ~ U(0.75, 1.25); num_batches_tracked = 0.
    (Golden fixtures overwrite the BN stats with calibrated ones.)
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    out = OrderedDict()
    for name, shape in param_shapes(cfg).items():
        if name.endswith("num_batches_tracked"):
            out[name] = np.zeros((), dtype=np.int64)
        elif name.endswith("running_mean"):
            out[name] = (0.1 * rng.standard_normal(shape)).astype(np.float32)
        elif name.endswith("running_var"):
            out[name] = rng.uniform(0.75, 1.25, shape).astype(np.float32)
        else:
            wname = name.rsplit(".", 1)[0] + ".weight"
            wshape = param_shapes(cfg)[wname]
            fan_in = int(np.prod(wshape[1:]))
            bound = 1.0 / math.sqrt(fan_in)
            out[name] = rng.uniform(-bound, bound, shape).astype(np.float32)
    return out


def params_checksum(params):
    """float64 sum of |p| and of p*index-weights, to detect PRNG drift."""
    s = 0.0
    t = 0.0
    for v in params.values():
        a = np.asarray(v, dtype=np.float64).ravel()
        s += float(np.abs(a).sum())
        t += float((a * (np.arange(a.size) % 7 + 1)).sum())
    return np.array([s, t], dtype=np.float64)


# --------------------------------------------------------------------------- #
# primitive ops
# --------------------------------------------------------------------------- #
def conv2d(x, w, b=None, stride=(1, 1), padding=(0, 0), dilation=(1, 1), acc=np.float64):
    """NCHW x OIHW cross-correlation, torch.nn.functional.conv2d semantics (zero padding)."""
    x = np.asarray(x, dtype=acc)
    w = np.asarray(w, dtype=acc)
    n, c, h, wd = x.shape
    o, ci, kh, kw = w.shape
    assert ci == c
    ph, pw = padding
    if ph or pw:
        x = np.pad(x, ((0, 0), (0, 0), (ph, ph), (pw, pw)))
    dh, dw = dilation
    sh, sw = stride
    eh, ew = dh * (kh - 1) + 1, dw * (kw - 1) + 1
    oh = (x.shape[2] - eh) // sh + 1
    ow = (x.shape[3] - ew) // sw + 1
    win = np.lib.stride_tricks.sliding_window_view(x, (eh, ew), axis=(2, 3))
    win = win[:, :, ::sh, ::sw, ::dh, ::dw][:, :, :oh, :ow]          # n c oh ow kh kw
    cols = np.ascontiguousarray(win.transpose(0, 2, 3, 1, 4, 5)).reshape(n * oh * ow, c * kh * kw)
    y = cols @ w.reshape(o, -1).T                                    # (n oh ow) o
    if b is not None:
        y = y + np.asarray(b, dtype=acc)
    return y.reshape(n, oh, ow, o).transpose(0, 3, 1, 2)


def relu(x):
    return np.maximum(x, 0)


def avg_pool2d(x, k):
    """nn.AvgPool2d(k) (stride=k, no padding, floor)."""
    kh, kw = k
    n, c, h, w = x.shape
    oh, ow = h // kh, w // kw
    x = x[:, :, : oh * kh, : ow * kw].reshape(n, c, oh, kh, ow, kw)
    return x.mean(axis=(3, 5))


def max_pool2d(x, k):
    """nn.MaxPool2d(k) (stride=k, no padding, floor)."""
    kh, kw = k
    n, c, h, w = x.shape
    oh, ow = h // kh, w // kw
    x = x[:, :, : oh * kh, : ow * kw].reshape(n, c, oh, kh, ow, kw)
    return x.max(axis=(3, 5))


def batch_norm_eval(x, mean, var, eps=1e-5):
    """BatchNorm2d(affine=False) in eval mode (model.py:100,118)."""
    mean = np.asarray(mean, dtype=x.dtype)[None, :, None, None]
    var = np.asarray(var, dtype=x.dtype)[None, :, None, None]
    return (x - mean) / np.sqrt(var + eps)


def linear(x, w, b):
    return x @ np.asarray(w, dtype=x.dtype).T + np.asarray(b, dtype=x.dtype)


# --------------------------------------------------------------------------- #
# forward passes
# --------------------------------------------------------------------------- #
def res_forward(params, cfg, x, acc=np.float64, trace=None):
    """SpeechResModel.forward, model.py:104-121.

    x: [B, 101, 40].  Returns logits [B, n_labels].
    trace: optional list receiving per-layer x after BN (pre-mean), for debugging.
    """
    x = np.asarray(x, dtype=acc)[:, None]                              # :105 unsqueeze(1)
    n_layers = int(cfg["n_layers"])
    old_x = None
    for i in range(n_layers + 1):                                       # :106
        if i == 0:
            y = relu(conv2d(x, params["conv0.weight"], padding=(1, 1), acc=acc))   # :107
            if "res_pool" in cfg:                                       # :109-110
                y = avg_pool2d(y, tuple(cfg["res_pool"]))
            old_x = y                                                   # :111
            x = y                                                       # :116
        else:
            d = res_dilation(cfg, i)
            y = relu(conv2d(x, params[f"conv{i}.weight"], padding=(d, d), dilation=(d, d), acc=acc))
            if i % 2 == 0:                                              # :112-114
                x = y + old_x
                old_x = x
            else:
                x = y
            x = batch_norm_eval(x, params[f"bn{i}.running_mean"], params[f"bn{i}.running_var"])  # :117-118
        if trace is not None:
            trace.append(x)
    x = x.reshape(x.shape[0], x.shape[1], -1).mean(axis=2)             # :119-120
    return linear(x, params["output.weight"], params["output.bias"])   # :121


def res_prebn_max(params, cfg, x):
    """max |value| over the tensors the packed res kernels store (conv0's output and
    every layer's pre-BN output, model.py:107-116), float64 -- the range an activation
    storage format must cover (tests/golden/make_range_golden.py)."""
    x = np.asarray(x, dtype=np.float64)[:, None]
    mx, old_x = 0.0, None
    for i in range(int(cfg["n_layers"]) + 1):
        if i == 0:
            y = relu(conv2d(x, params["conv0.weight"], padding=(1, 1)))
            if "res_pool" in cfg:
                y = avg_pool2d(y, tuple(cfg["res_pool"]))
            old_x = x = y
        else:
            d = res_dilation(cfg, i)
            y = relu(conv2d(x, params[f"conv{i}.weight"], padding=(d, d), dilation=(d, d)))
            x = y + old_x if i % 2 == 0 else y
            if i % 2 == 0:
                old_x = x
        mx = max(mx, float(np.nanmax(np.abs(x))))
        if i > 0:
            x = batch_norm_eval(x, params[f"bn{i}.running_mean"], params[f"bn{i}.running_var"])
    return mx


def cnn_forward(params, cfg, x, acc=np.float64):
    """SpeechModel.forward in eval mode (dropout = identity), model.py:186-205."""
    tf = bool(cfg.get("tf_variant"))
    x = np.asarray(x, dtype=acc)[:, None]
    x = relu(conv2d(x, params["conv1.weight"], params["conv1.bias"],
                    stride=tuple(cfg["conv1_stride"]), acc=acc))       # :187
    x = max_pool2d(x, tuple(cfg["conv1_pool"]))                         # :189
    if "conv2.weight" in params:                                        # :190-193
        x = relu(conv2d(x, params["conv2.weight"], params["conv2.bias"],
                        stride=tuple(cfg["conv2_stride"]), acc=acc))
        x = max_pool2d(x, tuple(cfg["conv2_pool"]))
    x = x.reshape(x.shape[0], -1)                                       # :194 (c,h,w) order
    if "lin.weight" in params:                                          # :195-196
        x = linear(x, params["lin.weight"], params["lin.bias"])
    if "dnn1.weight" in params:                                         # :197-201
        x = linear(x, params["dnn1.weight"], params["dnn1.bias"])
        if not tf:
            x = relu(x)
    if "dnn2.weight" in params:                                         # :202-204
        x = linear(x, params["dnn2.weight"], params["dnn2.bias"])
    return linear(x, params["output.weight"], params["output.bias"])   # :205


def calibrate_bn(params, cfg, xcal, shift=0.5, seed=0):
    """Set every bn{i} running stat from the pre-BN activations of ``xcal``.

    running_var = batch variance; running_mean = batch mean + shift*std*N(0,1)
    (per channel).  The shift leaves every BN output O(1) but with non-zero
    channel means, so the spatial mean that feeds the classifier (model.py:119-121)
    carries signal and logit parity actually exercises the conv stack.
    Returns a new params dict (float32 stats).
    """
    params = OrderedDict(params)
    rng = np.random.Generator(np.random.PCG64(seed))
    x = np.asarray(xcal, dtype=np.float64)[:, None]
    old_x = None
    for i in range(int(cfg["n_layers"]) + 1):
        if i == 0:
            y = relu(conv2d(x, params["conv0.weight"], padding=(1, 1)))
            if "res_pool" in cfg:
                y = avg_pool2d(y, tuple(cfg["res_pool"]))
            old_x = x = y
            continue
        d = res_dilation(cfg, i)
        y = relu(conv2d(x, params[f"conv{i}.weight"], padding=(d, d), dilation=(d, d)))
        if i % 2 == 0:
            x = y + old_x
            old_x = x
        else:
            x = y
        mean = x.mean(axis=(0, 2, 3))
        var = x.var(axis=(0, 2, 3)) + 1e-3
        mean = mean + shift * np.sqrt(var) * rng.standard_normal(mean.shape)
        params[f"bn{i}.running_mean"] = mean.astype(np.float32)
        params[f"bn{i}.running_var"] = var.astype(np.float32)
        x = batch_norm_eval(x, params[f"bn{i}.running_mean"], params[f"bn{i}.running_var"])
    return params


def forward(params, cfg, x, acc=np.float64):
    if "n_layers" in cfg:
        return res_forward(params, cfg, x, acc=acc)
    return cnn_forward(params, cfg, x, acc=acc)


def res_flops_per_clip(cfg, height=101, width=40):
    """Algorithmic FLOP per clip (2 x conv+linear MACs), SURVEY.md §8(d)."""
    c = int(cfg["n_feature_maps"])
    h, w = height, width
    macs = h * w * c * 9                       # conv0 at full resolution
    if "res_pool" in cfg:
        ph, pw = cfg["res_pool"]
        h, w = h // ph, w // pw
    macs += int(cfg["n_layers"]) * h * w * c * c * 9
    macs += c * int(cfg["n_labels"])
    return 2 * macs


def cnn_flops_per_clip(cfg):
    geo = cnn_geometry(cfg)
    macs = 0
    shapes = cnn_param_shapes(cfg)
    c1, oh, ow = geo["conv1"]
    macs += c1 * oh * ow * int(np.prod(shapes["conv1.weight"][1:]))
    if "conv2" in geo:
        c2, oh2, ow2 = geo["conv2"]
        macs += c2 * oh2 * ow2 * int(np.prod(shapes["conv2.weight"][1:]))
    for k in ("lin", "dnn1", "dnn2", "output"):
        if f"{k}.weight" in shapes:
            o, i = shapes[f"{k}.weight"]
            macs += o * i
    return 2 * macs


def flops_per_clip(cfg):
    return res_flops_per_clip(cfg) if "n_layers" in cfg else cnn_flops_per_clip(cfg)


# --------------------------------------------------------------------------- #
# training-set augmentation: SpeechDataset.load_audio's transform given its draws
# (model.py:282-306, _timeshift_audio :264-270), the same NumPy operations
# --------------------------------------------------------------------------- #
def timeshift(data, shift):
    """_timeshift_audio with the drawn shift (model.py:265-270)."""
    a = -min(0, shift)
    b = max(0, shift)
    data = np.pad(data, (a, b), "constant")
    return data[:len(data) - a] if a else data[b:]


def augment_clip(data, bg_slice, shift, amp, silence, mix, input_length, train=True):
    """load_audio after its draws (model.py:290-306): data the clip (float32; ignored
    for silence), bg_slice the drawn noise slice (float32, or None: np.zeros(input_length)
    as the reference uses without noise files), amp the drawn Python float a."""
    if bg_slice is None:
        bg_slice = np.zeros(input_length)
    if silence:
        data = np.zeros(input_length, dtype=np.float32)
    data = np.pad(data, (0, max(0, input_length - len(data))), "constant")
    if train:
        data = timeshift(data, shift)
    if mix:
        data = np.clip(amp * bg_slice + data, -1, 1)
    return data
