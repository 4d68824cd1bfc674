"""Generate the TRAINING golden fixtures (tests/golden/train_*.npz) by running the
reference's own training step.

Build container only (imports /root/reference, which never travels to the GPU
box); the same inert import stubs as make_golden.py.  Each case runs the
reference's ``SpeechResModel`` in train mode with the reference's optimizer and
step sequence (/root/reference/utils/train.py:99, :125-135):

    optimizer = torch.optim.SGD(model.parameters(), lr=lr, nesterov=..., weight_decay=wd, momentum=m)
    optimizer.zero_grad(); scores = model(x); loss = CrossEntropyLoss()(scores, y)
    loss.backward(); optimizer.step()

and records, per step: the loss, every parameter's gradient, every parameter
after the update, and the BN running statistics after the step.

``train_dp2_<model>.npz`` is the data-parallel (DDP) semantics of config C5 at
world size 2: the batch is split into two contiguous shards, each
shard runs forward/backward on its own copy of the model (per-replica BN batch
statistics), the gradients are averaged, and ONE SGD step is applied to the mean.
Running statistics are rank 0's (its shard's forward).

Weights come from ``oracle.ref_numpy.make_params`` (PCG64 seed) with BN running
stats from ``calibrate_bn``; inputs/labels from a PCG64 stream.  Usage:

    python tests/golden/make_train_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
from oracle import ref_numpy as orc  # noqa: E402

from make_golden import _stub_imports  # noqa: E402

CASES = [
    # name, model, batch, steps, lr, momentum, weight_decay, nesterov, seed
    ("train_res8-narrow", "res8-narrow", 6, 2, 0.1, 0.9, 1e-5, True, 301),
    ("train_res26-narrow", "res26-narrow", 4, 2, 0.1, 0.9, 1e-5, False, 302),
    ("train_res15-narrow", "res15-narrow", 3, 1, 0.01, 0.9, 1e-5, False, 303),
]
DP_CASES = [
    # name, model, batch (split in 2 shards), lr, momentum, weight_decay, nesterov, seed
    ("train_dp2_res26-narrow", "res26-narrow", 8, 0.1, 0.9, 1e-5, False, 304),
]
# Compact cases at the reference's own batch (utils/train.py:171 batch_size=64):
# inputs and labels are NOT stored -- they regenerate from the PCG64 seed (checked
# against the stored float64 sum / sum of squares) -- and parameters are stored
# after the last step only (every step's loss and gradients are stored).
# Overrides are merged into the reference config before the model is built; the cnn
# cases set dropout_prob = 0 so the step is RNG-free (dropout semantics are tested
# separately, on the device, against PyTorch's own dropout).
COMPACT_CASES = [
    # name, model, overrides, batch, steps, lr, momentum, weight_decay, nesterov, seed
    ("train_res26-narrow-b64", "res26-narrow", {}, 64, 2, 0.1, 0.9, 1e-5, False, 305),
    ("train_cnn-trad-pool2-b64", "cnn-trad-pool2", dict(dropout_prob=0.0), 64, 2, 0.01, 0.9, 1e-5, False, 306),
    ("train_cnn-one-fstride4-b64", "cnn-one-fstride4", dict(dropout_prob=0.0, n_labels=12), 64, 2, 0.01, 0.9,
     1e-5, True, 307),
]
COMPACT_DP_CASES = [
    # name, model, batch (split in 2 shards of 32), lr, momentum, weight_decay, nesterov, seed
    ("train_dp2_res26-narrow-b64", "res26-narrow", 64, 0.1, 0.9, 1e-5, False, 308),
]


def _model(mod, name, params):
    cfg = dict(mod.find_config(name))
    m = mod.find_model(name)(cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    return cfg, m


def _x_check(x):
    return np.array([float(np.sum(x, dtype=np.float64)), float(np.sum(np.square(x, dtype=np.float64)))])


def _inputs(seed, batch, n_labels):
    rng = np.random.Generator(np.random.PCG64(seed + 7000))
    x = rng.standard_normal((batch, 101, 40)).astype(np.float32)
    y = rng.integers(0, n_labels, size=batch).astype(np.int64)
    return x, y, rng


def _params(cfg, seed, rng):
    params = orc.make_params(cfg, seed)
    calib = rng.standard_normal((2, 101, 40)).astype(np.float32)
    return orc.calibrate_bn(params, cfg, calib, seed=seed)


def _buffers(m):
    return {k: v.detach().numpy().copy() for k, v in m.state_dict().items() if "running_" in k}


def main():
    _stub_imports()
    import utils.model as mod  # the reference
    torch.set_num_threads(8)
    crit = torch.nn.CrossEntropyLoss()

    for name, model_name, batch, steps, lr, mom, wd, nest, seed in CASES:
        cfg0 = dict(mod.find_config(model_name))
        x, y, rng = _inputs(seed, batch, cfg0["n_labels"])
        params = _params(cfg0, seed, rng)
        cfg, model = _model(mod, model_name, params)
        opt = torch.optim.SGD(model.parameters(), lr=lr, nesterov=nest, weight_decay=wd, momentum=mom)
        out = dict(model=np.array(model_name), seed=np.array(seed), x=x, y=y, lr=np.array(lr),
                   momentum=np.array(mom), weight_decay=np.array(wd), nesterov=np.array(nest),
                   steps=np.array(steps), keys=np.array([k for k, _ in model.named_parameters()]),
                   checksum=orc.params_checksum(params))
        for k, v in params.items():
            if "running_" in k:
                out[f"init__{k}"] = np.asarray(v, np.float32)
        losses = []
        for s in range(steps):
            model.train()
            opt.zero_grad()
            scores = model(torch.from_numpy(x))
            loss = crit(scores, torch.from_numpy(y))
            loss.backward()
            for k, p in model.named_parameters():
                out[f"g{s}__{k}"] = p.grad.detach().numpy().copy()
            opt.step()
            losses.append(float(loss.item()))
            for k, p in model.named_parameters():
                out[f"p{s}__{k}"] = p.detach().numpy().copy()
            for k, v in _buffers(model).items():
                out[f"b{s}__{k}"] = v
        out["loss"] = np.array(losses, np.float64)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        print(f"{name:26s} B={batch} steps={steps} losses={losses}")

    for name, model_name, batch, lr, mom, wd, nest, seed in DP_CASES:
        cfg0 = dict(mod.find_config(model_name))
        x, y, rng = _inputs(seed, batch, cfg0["n_labels"])
        params = _params(cfg0, seed, rng)
        half = batch // 2
        grads, losses, bufs0 = [], [], None
        for r in range(2):
            cfg, m = _model(mod, model_name, params)
            m.train()
            sl = slice(r * half, (r + 1) * half)
            loss = crit(m(torch.from_numpy(x[sl])), torch.from_numpy(y[sl]))
            loss.backward()
            grads.append({k: p.grad.detach().numpy().copy() for k, p in m.named_parameters()})
            losses.append(float(loss.item()))
            if r == 0:
                bufs0 = _buffers(m)
        cfg, m = _model(mod, model_name, params)
        opt = torch.optim.SGD(m.parameters(), lr=lr, nesterov=nest, weight_decay=wd, momentum=mom)
        opt.zero_grad()
        for k, p in m.named_parameters():
            p.grad = torch.from_numpy((grads[0][k] + grads[1][k]) / 2)
        opt.step()
        out = dict(model=np.array(model_name), seed=np.array(seed), x=x, y=y, lr=np.array(lr),
                   momentum=np.array(mom), weight_decay=np.array(wd), nesterov=np.array(nest),
                   keys=np.array([k for k, _ in m.named_parameters()]), checksum=orc.params_checksum(params),
                   shard_loss=np.array(losses, np.float64))
        for k, v in params.items():
            if "running_" in k:
                out[f"init__{k}"] = np.asarray(v, np.float32)
        for k, p in m.named_parameters():
            out[f"gmean__{k}"] = ((grads[0][k] + grads[1][k]) / 2).astype(np.float32)
            out[f"p0__{k}"] = p.detach().numpy().copy()
        for k, v in bufs0.items():
            out[f"b0__{k}"] = v
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        print(f"{name:26s} B={batch} shard losses={losses}")
    compact(mod, crit)


def compact(mod, crit):
    import json
    for name, model_name, over, batch, steps, lr, mom, wd, nest, seed in COMPACT_CASES:
        cfg0 = dict(mod.find_config(model_name))
        cfg0.update(over)
        x, y, rng = _inputs(seed, batch, cfg0["n_labels"])
        if "n_layers" in cfg0:
            params = _params(cfg0, seed, rng)
        else:
            params = orc.make_params(cfg0, seed)
        model = mod.find_model(model_name)(dict(cfg0))
        model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
        opt = torch.optim.SGD(model.parameters(), lr=lr, nesterov=nest, weight_decay=wd, momentum=mom)
        out = dict(model=np.array(model_name), overrides=np.array(json.dumps(over, sort_keys=True)),
                   seed=np.array(seed), batch=np.array(batch), x_check=_x_check(x),
                   y_check=np.array(int(np.sum(y * (np.arange(batch) + 1)))), lr=np.array(lr),
                   momentum=np.array(mom), weight_decay=np.array(wd), nesterov=np.array(nest), steps=np.array(steps),
                   keys=np.array([k for k, _ in model.named_parameters()]), checksum=orc.params_checksum(params))
        for k, v in params.items():
            if "running_" in k:
                out[f"init__{k}"] = np.asarray(v, np.float32)
        losses = []
        for s in range(steps):
            model.train()
            opt.zero_grad()
            loss = crit(model(torch.from_numpy(x)), torch.from_numpy(y))
            loss.backward()
            for k, p in model.named_parameters():
                out[f"g{s}__{k}"] = p.grad.detach().numpy().copy()
            opt.step()
            losses.append(float(loss.item()))
            if s == steps - 1:
                for k, p in model.named_parameters():
                    out[f"p{s}__{k}"] = p.detach().numpy().copy()
            for k, v in _buffers(model).items():
                out[f"b{s}__{k}"] = v
        out["loss"] = np.array(losses, np.float64)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        print(f"{name:30s} B={batch} steps={steps} losses={losses}")

    for name, model_name, batch, lr, mom, wd, nest, seed in COMPACT_DP_CASES:
        cfg0 = dict(mod.find_config(model_name))
        x, y, rng = _inputs(seed, batch, cfg0["n_labels"])
        params = _params(cfg0, seed, rng)
        half = batch // 2
        grads, losses, bufs0 = [], [], None
        for r in range(2):
            cfg, m = _model(mod, model_name, params)
            m.train()
            sl = slice(r * half, (r + 1) * half)
            loss = crit(m(torch.from_numpy(x[sl])), torch.from_numpy(y[sl]))
            loss.backward()
            grads.append({k: p.grad.detach().numpy().copy() for k, p in m.named_parameters()})
            losses.append(float(loss.item()))
            if r == 0:
                bufs0 = _buffers(m)
        cfg, m = _model(mod, model_name, params)
        opt = torch.optim.SGD(m.parameters(), lr=lr, nesterov=nest, weight_decay=wd, momentum=mom)
        opt.zero_grad()
        for k, p in m.named_parameters():
            p.grad = torch.from_numpy((grads[0][k] + grads[1][k]) / 2)
        opt.step()
        out = dict(model=np.array(model_name), overrides=np.array("{}"), seed=np.array(seed), batch=np.array(batch),
                   x_check=_x_check(x), y_check=np.array(int(np.sum(y * (np.arange(batch) + 1)))), lr=np.array(lr),
                   momentum=np.array(mom), weight_decay=np.array(wd), nesterov=np.array(nest),
                   keys=np.array([k for k, _ in m.named_parameters()]), checksum=orc.params_checksum(params),
                   shard_loss=np.array(losses, np.float64))
        for k, v in params.items():
            if "running_" in k:
                out[f"init__{k}"] = np.asarray(v, np.float32)
        for k, p in m.named_parameters():
            out[f"gmean__{k}"] = ((grads[0][k] + grads[1][k]) / 2).astype(np.float32)
            out[f"p0__{k}"] = p.detach().numpy().copy()
        for k, v in bufs0.items():
            out[f"b0__{k}"] = v
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        print(f"{name:30s} B={batch} shard losses={losses}")


if __name__ == "__main__":
    main()
