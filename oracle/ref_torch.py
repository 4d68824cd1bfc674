"""Oracle, torch-CPU form: the same restatement as ``ref_numpy`` on stock
``torch.nn.functional`` ops in fp32 -- what the reference's own CPU path
(``utils/train.py --no_cuda``: torch eval forward on the host) executes.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (``honk_amd``) imports this
module; ``bench.py``'s ``cpu_baseline`` leg times it on the host cores, and
``tests/test_oracle_golden.py`` pins it against the reference-generated
fixtures in ``tests/golden/`` (fp32: 1e-5 absolute, like ``ref_numpy``'s fp32 path).

* ``SpeechResModel.forward`` -- /root/reference/utils/model.py:104-121
* ``SpeechModel.forward``    -- /root/reference/utils/model.py:186-205
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from oracle.ref_numpy import res_dilation


def _t(params, k):
    v = params[k]
    return v if isinstance(v, torch.Tensor) else torch.as_tensor(v, dtype=torch.float32)


def tensors(params):
    """numpy params -> fp32 torch tensors (once per model)."""
    return {k: _t(params, k).float() for k in params}


def res_forward(p, cfg, x):
    """model.py:104-121: conv0 (+pool) then n_layers dilated 3x3 convs, ReLU,
    pre-BN residual on even layers, BatchNorm (eval), spatial mean, Linear."""
    x = x.unsqueeze(1)                                                     # :105
    old_x = None
    for i in range(int(cfg["n_layers"]) + 1):                               # :106
        if i == 0:
            y = F.relu(F.conv2d(x, p["conv0.weight"], padding=1))           # :107
            if "res_pool" in cfg:                                           # :109-110
                y = F.avg_pool2d(y, tuple(cfg["res_pool"]))
            old_x = x = y                                                   # :111,116
            continue
        d = res_dilation(cfg, i)
        y = F.relu(F.conv2d(x, p[f"conv{i}.weight"], padding=d, dilation=d))
        if i % 2 == 0:                                                      # :112-114
            x = y + old_x
            old_x = x
        else:
            x = y
        x = F.batch_norm(x, p[f"bn{i}.running_mean"], p[f"bn{i}.running_var"], training=False)  # :117-118
    x = x.reshape(x.shape[0], x.shape[1], -1).mean(2)                      # :119-120
    return F.linear(x, p["output.weight"], p["output.bias"])               # :121


def cnn_forward(p, cfg, x):
    """model.py:186-205 in eval mode (dropout = identity)."""
    tf = bool(cfg.get("tf_variant"))
    x = x.unsqueeze(1)
    x = F.relu(F.conv2d(x, p["conv1.weight"], p["conv1.bias"], stride=tuple(cfg["conv1_stride"])))  # :187
    x = F.max_pool2d(x, tuple(cfg["conv1_pool"]))                           # :189
    if "conv2.weight" in p:                                                 # :190-193
        x = F.relu(F.conv2d(x, p["conv2.weight"], p["conv2.bias"], stride=tuple(cfg["conv2_stride"])))
        x = F.max_pool2d(x, tuple(cfg["conv2_pool"]))
    x = x.reshape(x.shape[0], -1)                                           # :194
    if "lin.weight" in p:                                                   # :195-196
        x = F.linear(x, p["lin.weight"], p["lin.bias"])
    if "dnn1.weight" in p:                                                  # :197-201
        x = F.linear(x, p["dnn1.weight"], p["dnn1.bias"])
        if not tf:
            x = F.relu(x)
    if "dnn2.weight" in p:                                                  # :202-204
        x = F.linear(x, p["dnn2.weight"], p["dnn2.bias"])
    return F.linear(x, p["output.weight"], p["output.bias"])               # :205


@torch.no_grad()
def forward(params, cfg, x):
    """Logits [B, n_labels] (fp32) for x [B, 101, 40] (numpy or CPU tensor)."""
    p = params if all(isinstance(v, torch.Tensor) for v in params.values()) else tensors(params)
    x = x if isinstance(x, torch.Tensor) else torch.as_tensor(x, dtype=torch.float32)
    if "n_layers" in cfg:
        return res_forward(p, cfg, x.float())
    return cnn_forward(p, cfg, x.float())
