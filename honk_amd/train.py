"""Callers of the hot path: the evaluate()/train() surface of /root/reference/utils/train.py.

Behaviour (console format, config keys, SGD/LR-schedule semantics, optimizer
re-creation quirk) follows the reference; the model comes from
``config["model_class"]`` exactly as there, so a ``honk_amd.model`` class runs
its forward on the gfx950 kernels whenever the model is on a ROCm device in
eval mode.

Differences, both additive: ``evaluate``/``train`` accept injected loaders /
datasets (the reference builds them from ``SpeechDataset.splits``, which needs
the Speech Commands folders and librosa -- out of scope); a
``honk_amd.data.DeviceSpeechDataset`` is consumed on the device (its batches are
clip indices: ``load_audio``'s augmentation and ``collate_fn``'s MFCCs run as
kernels, honk_amd/data.py).
"""
from __future__ import annotations

import argparse
import copy
import os
import random
from collections import ChainMap

import numpy as np
import torch
import torch.nn as nn
import torch.utils.data as data

from . import distributed as hd
from . import syncbn
from . import head_train
from .data import batch_input
from . import model as mod
from .optim import FlatParams, FlatSGD


class ConfigBuilder(object):
    """utils/train.py:17-39: one ``--flag`` per default-config key."""

    def __init__(self, *default_configs):
        self.default_config = ChainMap(*default_configs)

    def build_argparse(self):
        parser = argparse.ArgumentParser()
        for key, value in self.default_config.items():
            flag = "--" + key
            if isinstance(value, tuple):
                parser.add_argument(flag, default=list(value), nargs=len(value), type=type(value[0]))
            elif isinstance(value, list):
                parser.add_argument(flag, default=value, nargs="+", type=type(value[0]))
            elif isinstance(value, bool) and not value:
                parser.add_argument(flag, action="store_true")
            else:
                parser.add_argument(flag, default=value, type=type(value))
        return parser

    def config_from_argparse(self, parser=None):
        parser = parser or self.build_argparse()
        args = vars(parser.parse_known_args()[0])
        return ChainMap(args, self.default_config)


def print_eval(name, scores, labels, loss, end="\n"):
    """utils/train.py:41-46: top-1 accuracy of the batch; prints and returns it."""
    n = labels.size(0)
    pred = torch.max(scores, 1)[1].view(n)
    accuracy = (pred.data == labels.data).float().sum() / n
    print("{} accuracy: {:>5}, loss: {:<25}".format(name, accuracy, loss.item()), end=end)
    return accuracy.item()


def set_seed(config):
    """utils/train.py:48-54."""
    seed = config["seed"]
    torch.manual_seed(seed)
    np.random.seed(seed)
    if not config["no_cuda"]:
        torch.cuda.manual_seed(seed)
    random.seed(seed)


def _select_device(config):
    """utils/train.py:64,70,97: ``torch.cuda.set_device(config["gpu_no"])``.  In a
    one-process-per-GPU job (torch.distributed up with world > 1) each rank takes
    its own device (LOCAL_RANK) instead, so the replicas do not share one GPU."""
    if not config["no_cuda"]:
        torch.cuda.set_device(hd.local_device_index(config["gpu_no"]))


def _whole_set_loader(dataset):
    return data.DataLoader(dataset, batch_size=len(dataset), shuffle=False,
                           collate_fn=getattr(dataset, "collate_fn", None))


def evaluate(config, model=None, test_loader=None):
    """utils/train.py:56-85: whole test set as one batch, prints per-batch and final accuracy."""
    if not test_loader:
        _, _, test_set = mod_splits(config)
        test_loader = _whole_set_loader(test_set)
    _select_device(config)
    if not model:
        model = config["model_class"](config)
        model.load(config["input_file"])
    if not config["no_cuda"]:
        _select_device(config)
        model.cuda()
    model.eval()
    criterion = nn.CrossEntropyLoss()
    weighted, total = [], 0
    with torch.no_grad():
        for model_in, labels in test_loader:
            model_in = batch_input(test_loader.dataset, model_in)  # device datasets: indices -> MFCCs
            if not config["no_cuda"]:
                model_in, labels = model_in.cuda(), labels.cuda()
            scores = model(model_in)
            loss = criterion(scores, labels)
            weighted.append(print_eval("test", scores, labels, loss) * model_in.size(0))
            total += model_in.size(0)
    print("final test accuracy: {}".format(sum(weighted) / total))


def mod_splits(config):
    splits = getattr(mod, "SpeechDataset", None)
    if splits is None:
        raise RuntimeError("honk_amd: dataset loading (SpeechDataset.splits) is out of scope; "
                           "pass test_loader= / datasets= explicitly")
    return splits.splits(config)


def _sgd(flat, config, lr):
    return FlatSGD(flat, lr=lr, momentum=config["momentum"], weight_decay=config["weight_decay"],
                   nesterov=config["use_nesterov"])


def train(config, datasets=None):
    """utils/train.py:87-163: SGD training with the reference's schedule semantics.

    ``schedule`` step thresholds switch to ``lr[i]`` by RE-CREATING the optimizer
    (momentum buffers reset, :137-141); dev evaluation every ``dev_every``
    epochs keeps the best model (saved to ``output_file``); the best model is
    evaluated on the test set at the end.

    Optimizer: FlatSGD (torch.optim.SGD semantics over one flat bucket; fused
    HIP kernel on ROCm).  When torch.distributed is initialised with world > 1
    this is data-parallel with DDP semantics: each rank
    draws ``batch_size`` clips per step from its shard of the train set, BN uses
    per-replica batch statistics with running stats broadcast from rank 0 (ONE
    broadcast of the flat buffer bucket per step), the gradient bucket is summed
    with ONE all-reduce -- started from the hook of the last gradient backward
    writes -- and averaged in the SGD kernel: two collectives per step.  Only rank
    0 prints and saves.  ``sync_bn`` (or HONK_SYNC_BN=1): SyncBN instead of the
    per-replica statistics, one more all-reduce per BatchNorm and direction
    (honk_amd/syncbn.py).
    """
    rank, world = hd.world_info()
    log = rank == 0
    out_dir = os.path.dirname(os.path.abspath(config["output_file"]))
    if log:
        os.makedirs(out_dir, exist_ok=True)
    train_set, dev_set, test_set = datasets if datasets is not None else mod_splits(config)
    model = config["model_class"](config)
    if config["input_file"]:
        model.load(config["input_file"])
    if not config["no_cuda"]:
        _select_device(config)
        model.cuda()
    hd.broadcast_module(model)
    flat = FlatParams(model)
    fbuf = hd.FlatBuffers(model)     # BN running stats: one broadcast per step
    reducer = hd.GradAllReduce(flat)  # grads: one all-reduce per step, started by backward
    optimizer = _sgd(flat, config, config["lr"][0])
    schedule_steps = config["schedule"]  # the caller's list, extended in place (utils/train.py:100-101)
    schedule_steps.append(np.inf)
    criterion = head_train.CrossEntropyLoss()  # nn.CrossEntropyLoss(); native on ROCm tensors

    if world > 1:
        sampler = data.distributed.DistributedSampler(train_set, num_replicas=world, rank=rank, shuffle=True,
                                                      seed=int(config["seed"]), drop_last=True)
        train_loader = data.DataLoader(train_set, batch_size=config["batch_size"], sampler=sampler, drop_last=True,
                                       collate_fn=getattr(train_set, "collate_fn", None))
    else:
        sampler = None
        train_loader = data.DataLoader(train_set, batch_size=config["batch_size"], shuffle=True, drop_last=True,
                                       collate_fn=getattr(train_set, "collate_fn", None))
    dev_loader = data.DataLoader(dev_set, batch_size=min(len(dev_set), 16), shuffle=False,
                                 collate_fn=getattr(dev_set, "collate_fn", None))
    test_loader = _whole_set_loader(test_set)
    # optional SyncBN (config["sync_bn"] or HONK_SYNC_BN=1; honk_amd/syncbn.py): the
    # train-mode BatchNorms normalise with the whole job's statistics instead of the shard's
    sync = world > 1 and bool(config.get("sync_bn", os.environ.get("HONK_SYNC_BN", "0") == "1"))
    if sync:
        syncbn.enable()
    try:
        best_model = _train_epochs(config, model, train_set, dev_set, train_loader, dev_loader, sampler, flat,
                                   fbuf, reducer, optimizer, schedule_steps, criterion, log)
    finally:
        reducer.remove()  # no gradient hooks (and no stray all-reduce) outlive train()
        if sync:
            syncbn.disable()
    if log:
        evaluate(config, best_model, test_loader)


def _train_epochs(config, model, train_set, dev_set, train_loader, dev_loader, sampler, flat, fbuf, reducer,
                  optimizer, schedule_steps, criterion, log):
    """utils/train.py:123-162: the epochs of train(); returns the best model on dev."""
    sched_idx, step_no, max_acc, best_model = 0, 0, 0, None
    for epoch_idx in range(config["n_epochs"]):
        if sampler is not None:
            sampler.set_epoch(epoch_idx)
        for model_in, labels in train_loader:
            model.train()
            optimizer.zero_grad()
            reducer.reset()
            labels_host = labels
            # a DeviceSpeechDataset batch is clip indices: augmentation + MFCC on the device
            model_in = batch_input(train_set, model_in)
            if not config["no_cuda"]:
                model_in, labels = model_in.cuda(), labels.cuda()
            hd.broadcast_buffers(fbuf)
            scores = model(model_in)
            head_train.check_labels(labels_host, scores.shape[1])  # torch's IndexError, on the host copy
            loss = criterion(scores, labels, labels_checked=True)
            loss.backward()
            optimizer.step(grad_scale=reducer.wait())
            step_no += 1
            if step_no > schedule_steps[sched_idx]:
                sched_idx += 1
                if log:
                    print("changing learning rate to {}".format(config["lr"][sched_idx]))
                optimizer = _sgd(flat, config, config["lr"][sched_idx])
            if log:
                print_eval("train step #{}".format(step_no), scores, labels, loss)

        if epoch_idx % config["dev_every"] == config["dev_every"] - 1:
            model.eval()
            accs = []
            with torch.no_grad():
                for model_in, labels in dev_loader:
                    model_in = batch_input(dev_set, model_in)
                    if not config["no_cuda"]:
                        model_in, labels = model_in.cuda(), labels.cuda()
                    scores = model(model_in)
                    loss = criterion(scores, labels)
                    if log:
                        accs.append(print_eval("dev", scores, labels, loss))
                    else:
                        accs.append(((scores.argmax(1) == labels).float().mean()).item())
            avg_acc = np.mean(accs)
            if log:
                print("final dev accuracy: {}".format(avg_acc))
            if avg_acc > max_acc:
                max_acc = avg_acc
                if log:
                    print("saving best model...")
                    model.save(config["output_file"])
                best_model = copy.deepcopy(model)
    return best_model


def default_run_config(output_file=None):
    """utils/train.py:171-172 run defaults."""
    if output_file is None:
        output_file = os.path.join(os.getcwd(), "model", "model.pt")
    return dict(no_cuda=False, n_epochs=500, lr=[0.001], schedule=[np.inf], batch_size=64, dev_every=10, seed=0,
                use_nesterov=False, input_file="", output_file=output_file, gpu_no=1, cache_size=32768,
                momentum=0.9, weight_decay=0.00001)


def dataset_default_config():
    """utils/model.py:234-251 SpeechDataset.default_config (keys only consumed by data loading)."""
    return dict(group_speakers_by_id=True, silence_prob=0.1, noise_prob=0.8, n_dct_filters=40, input_length=16000,
                n_mels=40, timeshift_ms=100, unknown_prob=0.1, train_pct=80, dev_pct=10, test_pct=10,
                wanted_words=["command", "random"], data_folder="/data/speech_dataset",
                audio_preprocess_type="MFCCs")


def main():
    """utils/train.py:165-186 CLI: ``python -m honk_amd.train --model res15 --type eval ...``."""
    parser = argparse.ArgumentParser()
    parser.add_argument("--model", choices=[x.value for x in list(mod.ConfigType)], default="cnn-trad-pool2",
                        type=str)
    config, _ = parser.parse_known_args()
    mod_cls = mod.find_model(config.model)
    builder = ConfigBuilder(mod.find_config(config.model), dataset_default_config(), default_run_config())
    parser = builder.build_argparse()
    parser.add_argument("--type", choices=["train", "eval"], default="train", type=str)
    config = builder.config_from_argparse(parser)
    config["model_class"] = mod_cls
    set_seed(config)
    if config["type"] == "train":
        train(config)
    elif config["type"] == "eval":
        evaluate(config)


if __name__ == "__main__":
    main()
