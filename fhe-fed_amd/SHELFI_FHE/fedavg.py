"""Encrypted FedAvg over model state dicts — the host-side flow of the reference's
harnesses, on top of the SHELFI_FHE API.

Restates (paths relative to /root/reference/code):
  * benchmark.py:16-29 / function_helper.py:7-26 — flatten a state_dict per key to
    float64 numpy vectors and back (`flatten_state`, `unflatten_state`);
  * benchmark.py:473-532 — weights 1/N, per key x client `encrypt`, per key
    `computeWeightedAverage`, per key `decrypt` to the layer size, with the timing
    boundaries printed at :539-543 (`SecureFedAvg.run`);
  * benchmark_selection.py:42-44,152-158 — encrypt only the keys whose layer index
    (the digits of the key) is selected, plain FedAvg for the rest (`select="layers"`);
  * benchmark_selection_rate.py:138-139,169 — encrypt the first round(len * rate)
    entries of every key, plain FedAvg for the rest (`select="rate"`);
  * attack/masking/masking.py:15-21 — a boolean sensitivity mask per key (top-k),
    encrypting only the masked entries (`select="mask"`).

`pack=True` concatenates all encrypted entries of a client into one vector before
encryption (one `encrypt` and one `computeWeightedAverage` per round instead of one
per key; the reference pads every key to whole ciphertexts).
"""
from __future__ import annotations

import re
import time
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence

import numpy as np


# ------------------------------------------------------------ state dicts --
def flatten_state(state) -> "OrderedDict[str, np.ndarray]":
    """benchmark.py:16-21 tensor_to_numpy_arr (float64, as py::array_t<double> forcecast)."""
    out = OrderedDict()
    for k, v in state.items():
        a = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
        out[k] = np.ascontiguousarray(a.reshape(-1), dtype=np.float64)
    return out


def state_shapes(state) -> "OrderedDict[str, tuple]":
    """function_helper.py:22-26 tensorShape."""
    return OrderedDict((k, tuple(v.shape)) for k, v in state.items())


def unflatten_state(params: Dict[str, np.ndarray], shapes: Dict[str, tuple], like=None):
    """benchmark.py:23-29 numpy_arr_to_tensor (torch tensors if torch is importable)."""
    try:
        import torch
    except ImportError:  # pragma: no cover
        torch = None
    out = OrderedDict()
    for k, v in params.items():
        arr = np.asarray(v).reshape(shapes[k])
        if torch is not None:
            t = torch.from_numpy(np.ascontiguousarray(arr))
            if like is not None and k in like and hasattr(like[k], "dtype"):
                t = t.to(like[k].dtype)
            out[k] = t
        else:
            out[k] = arr
    return out


def layer_index(key: str) -> Optional[int]:
    """benchmark_selection.py:42,152: the layer number is the key's digits."""
    d = re.sub("[^0-9]", "", key)
    return int(d) if d else None


def plain_fedavg(flat_states: Sequence[Dict[str, np.ndarray]], weights: Sequence[float], key: str,
                 idx=None) -> np.ndarray:
    acc = None
    for st, w in zip(flat_states, weights):
        x = st[key] if idx is None else st[key][idx]
        acc = w * x if acc is None else acc + w * x
    return acc


# --------------------------------------------------------------- selection --
class Selection:
    """Which entries of each key are encrypted.  mode:
    "all" (benchmark.py), "layers" (benchmark_selection.py: `layers` = set of layer
    indices), "rate" (benchmark_selection_rate.py: prefix fraction `rate`), "mask"
    (masking.py: `masks[key]` boolean arrays)."""

    def __init__(self, mode: str = "all", layers=None, rate: float = 1.0, masks=None):
        if mode not in ("all", "layers", "rate", "mask"):
            raise ValueError("unknown selection mode %r" % mode)
        self.mode, self.layers, self.rate, self.masks = mode, set(layers or ()), float(rate), masks or {}

    def encrypted_index(self, key: str, n: int):
        """None = nothing encrypted; slice/bool array of the encrypted entries."""
        if self.mode == "all":
            return slice(0, n)
        if self.mode == "layers":
            li = layer_index(key)
            return slice(0, n) if li is not None and li in self.layers else None
        if self.mode == "rate":
            cut = int(round(n * self.rate))  # benchmark_selection_rate.py:138
            return slice(0, cut) if cut > 0 else None
        m = self.masks.get(key)
        if m is None or not np.any(m):
            return None
        return np.asarray(m, dtype=bool).reshape(-1)


def top_k_mask(sensitivity: np.ndarray, fraction: float) -> np.ndarray:
    """masking.py:15-21 get_top_k_mask: True on the k = int(len(vector) * p) largest entries
    (`torch.topk(vector, int(len(vector) * p), largest=True)`: the product truncates, so the
    count is the floor of n * p).  The reference's Mask is the complement (False marks the
    protected entries, masking.py:19-20); here True marks the entries that get encrypted.
    Among equal values torch.topk's choice is unspecified, so is this one's."""
    s = np.asarray(sensitivity).reshape(-1)
    k = int(s.size * fraction)
    mask = np.zeros(s.size, dtype=bool)
    if k > 0:
        mask[np.argpartition(-s, k - 1)[:k]] = True
    return mask


# -------------------------------------------------------------- the round --
class SecureFedAvg:
    """One encrypted FedAvg round (benchmark.py:447-543) through a SHELFI_FHE.CKKS."""

    def __init__(self, ckks, selection: Optional[Selection] = None, pack: bool = False):
        self.ckks = ckks
        self.sel = selection or Selection("all")
        self.pack = pack
        self.times = {}

    def run(self, client_states: Sequence, weights: Optional[Sequence[float]] = None):
        """-> (aggregated flat params OrderedDict[key] -> float64 array, timings)."""
        N = len(client_states)
        if weights is None:
            weights = np.full(N, 1 / N).tolist()  # benchmark.py:473
        flats = [s if isinstance(next(iter(s.values())), np.ndarray) and next(iter(s.values())).ndim == 1
                 else flatten_state(s) for s in client_states]
        keys = list(flats[0].keys())
        plan = OrderedDict((k, self.sel.encrypted_index(k, flats[0][k].size)) for k in keys)
        result = OrderedDict()
        t = {"encrypt": 0.0, "aggregate": 0.0, "decrypt": 0.0, "plain": 0.0}

        # plaintext FedAvg of everything not encrypted (plain_aggregate in the harnesses)
        t0 = time.time()
        for k in keys:
            result[k] = plain_fedavg(flats, weights, k)
        t["plain"] = time.time() - t0

        enc_keys = [k for k in keys if plan[k] is not None]
        if not enc_keys:
            self.times = t
            return result, t
        if self.pack:
            sel_vecs = [np.concatenate([f[k][plan[k]] for k in enc_keys]) for f in flats]
            t0 = time.time()
            encs = [self.ckks.encrypt(v) for v in sel_vecs]
            t["encrypt"] = (time.time() - t0) / N  # benchmark.py:497 (per client)
            t0 = time.time()
            agg = self.ckks.computeWeightedAverage(encs, weights)
            t["aggregate"] = time.time() - t0
            t0 = time.time()
            dec = self.ckks.decrypt(agg, sel_vecs[0].size)
            t["decrypt"] = time.time() - t0
            off = 0
            for k in enc_keys:
                n = flats[0][k][plan[k]].size
                result[k][plan[k]] = dec[off:off + n]
                off += n
        else:
            encs: List[Dict[str, bytes]] = [dict() for _ in range(N)]
            t0 = time.time()
            for k in enc_keys:  # benchmark.py:489-494: per key x client
                for i in range(N):
                    encs[i][k] = self.ckks.encrypt(flats[i][k][plan[k]])
            t["encrypt"] = (time.time() - t0) / N
            t0 = time.time()
            aggs = {k: self.ckks.computeWeightedAverage([encs[i][k] for i in range(N)], weights)
                    for k in enc_keys}  # benchmark.py:506-514
            t["aggregate"] = time.time() - t0
            t0 = time.time()
            for k in enc_keys:  # benchmark.py:527-529
                n = flats[0][k][plan[k]].size
                result[k][plan[k]] = self.ckks.decrypt(aggs[k], n)
            t["decrypt"] = time.time() - t0
        self.times = t
        return result, t

    def report(self) -> str:
        """benchmark.py:539-543 prints."""
        t = self.times
        return ("Plaintext Time: {}\nEncryption Time: {}\nSecure Agg Time: {}\nDecryption Time: {}"
                .format(t.get("plain"), t.get("encrypt"), t.get("aggregate"), t.get("decrypt")))


# ------------------------------------------------------- synthetic models --
def resnet_shapes(depth: int = 18, num_classes: int = 1000, buffers: bool = True) -> "OrderedDict[str, tuple]":
    """torchvision ResNet-18/50 `model.state_dict()` shapes, in state_dict order: what
    benchmark.py:457 encrypts (tensor_to_numpy_arr(model.state_dict()), :16-21).  Every BatchNorm
    contributes weight, bias and the buffers running_mean, running_var and num_batches_tracked
    (a 0-d int64 tensor, flattened to one element); 20 BNs in ResNet-18, 53 in ResNet-50.
    buffers=False keeps the parameters alone (model.parameters(): 11,689,512 / 25,557,032)."""
    shapes = OrderedDict()

    def bn(prefix, c):
        shapes[prefix + "weight"] = (c,)
        shapes[prefix + "bias"] = (c,)
        if buffers:
            shapes[prefix + "running_mean"] = (c,)
            shapes[prefix + "running_var"] = (c,)
            shapes[prefix + "num_batches_tracked"] = ()

    shapes["conv1.weight"] = (64, 3, 7, 7)
    bn("bn1.", 64)
    if depth == 18:
        blocks, expansion = [2, 2, 2, 2], 1
    elif depth == 50:
        blocks, expansion = [3, 4, 6, 3], 4
    else:
        raise ValueError("depth 18 or 50")
    inplanes = 64
    for li, (planes, nb) in enumerate(zip([64, 128, 256, 512], blocks), start=1):
        for bi in range(nb):
            p = "layer%d.%d." % (li, bi)
            stride = 2 if (bi == 0 and li > 1) else 1
            if depth == 18:
                shapes[p + "conv1.weight"] = (planes, inplanes, 3, 3)
                bn(p + "bn1.", planes)
                shapes[p + "conv2.weight"] = (planes, planes, 3, 3)
                bn(p + "bn2.", planes)
                out = planes
            else:
                shapes[p + "conv1.weight"] = (planes, inplanes, 1, 1)
                bn(p + "bn1.", planes)
                shapes[p + "conv2.weight"] = (planes, planes, 3, 3)
                bn(p + "bn2.", planes)
                shapes[p + "conv3.weight"] = (planes * 4, planes, 1, 1)
                bn(p + "bn3.", planes * 4)
                out = planes * 4
            if bi == 0 and (stride != 1 or inplanes != out):
                shapes[p + "downsample.0.weight"] = (out, inplanes, 1, 1)
                bn(p + "downsample.1.", out)
            inplanes = out
    shapes["fc.weight"] = (num_classes, 512 * expansion)
    shapes["fc.bias"] = (num_classes,)
    return shapes


def cts_per_key(shapes, batch: int) -> "OrderedDict[str, int]":
    """Ciphertexts encrypt() makes per state_dict key (benchmark.py:490-493 encrypts each key on
    its own; ckks.cpp:65-83 chunks n values into ceil(n / batch), a 1-element buffer included)."""
    return OrderedDict((k, -(-max(1, int(np.prod(shp))) // batch)) for k, shp in shapes.items())


def lenet5_shapes() -> "OrderedDict[str, tuple]":
    """LeNet-5 (61,706 params; BASELINE config 2)."""
    return OrderedDict([("conv1.weight", (6, 1, 5, 5)), ("conv1.bias", (6,)),
                        ("conv2.weight", (16, 6, 5, 5)), ("conv2.bias", (16,)),
                        ("fc1.weight", (120, 400)), ("fc1.bias", (120,)),
                        ("fc2.weight", (84, 120)), ("fc2.bias", (84,)),
                        ("fc3.weight", (10, 84)), ("fc3.bias", (10,))])


def synthetic_states(shapes, num_clients: int, seed: int = 0, scale: float = 0.1):
    """Client state dicts flattened per key (tensor_to_numpy_arr, benchmark.py:16-21): float32
    weights U(-scale, scale) widened to float64; BatchNorm running_var U(0, 2 scale) (positive);
    num_batches_tracked an int64 step count (kept int64: encrypt's forcecast widens it, as the
    reference's py::array_t<double> does)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(num_clients):
        st = OrderedDict()
        for k, shp in shapes.items():
            n = int(np.prod(shp))
            if k.endswith("num_batches_tracked"):
                st[k] = rng.integers(0, 100_000, n, dtype=np.int64)
            elif k.endswith("running_var"):
                st[k] = rng.uniform(0, 2 * scale, n).astype(np.float32).astype(np.float64)
            else:
                st[k] = rng.uniform(-scale, scale, n).astype(np.float32).astype(np.float64)
        out.append(st)
    return out
