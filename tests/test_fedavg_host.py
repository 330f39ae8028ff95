"""CPU tests of the FedAvg harness host logic (SHELFI_FHE.fedavg): model shapes,
selection rules of benchmark_selection*.py / masking.py, flatten/unflatten."""
import numpy as np
import pytest

from SHELFI_FHE import fedavg as F


def test_model_param_counts():
    assert sum(int(np.prod(s)) for s in F.resnet_shapes(18, buffers=False).values()) == 11_689_512
    assert sum(int(np.prod(s)) for s in F.resnet_shapes(50, buffers=False).values()) == 25_557_032
    assert sum(int(np.prod(s)) for s in F.lenet5_shapes().values()) == 61_706


def _bn_channels(depth):
    """Independent count of BatchNorm channels in torchvision's ResNets: the stem's bn1, every
    block's BNs (2 of `planes` for BasicBlock; planes, planes, 4 planes for Bottleneck) and the
    first block's downsample BN of each stage that changes shape."""
    planes, blocks = [64, 128, 256, 512], {18: [2, 2, 2, 2], 50: [3, 4, 6, 3]}[depth]
    ch, n_bn = 64, 1
    for i, (p, nb) in enumerate(zip(planes, blocks)):
        per_block = [p, p] if depth == 18 else [p, p, 4 * p]
        ch += nb * sum(per_block)
        n_bn += nb * len(per_block)
        if depth == 50 or i > 0:  # stage 1 of ResNet-18 keeps 64 channels at stride 1: no downsample
            ch += per_block[-1]
            n_bn += 1
    return ch, n_bn


@pytest.mark.parametrize("depth,params,keys", [(18, 11_689_512, 62), (50, 25_557_032, 161)])
def test_state_dict_includes_batchnorm_buffers(depth, params, keys):
    """benchmark.py:457 encrypts model.state_dict(): every BN's running_mean, running_var and
    num_batches_tracked (one int64 element) ride along with the parameters, each its own key."""
    sh = F.resnet_shapes(depth)
    ch, n_bn = _bn_channels(depth)
    assert n_bn == {18: 20, 50: 53}[depth]
    assert len(sh) == keys + 3 * n_bn
    assert sum(int(np.prod(s)) for s in sh.values()) == params + 2 * ch + n_bn
    nbt = [k for k in sh if k.endswith("num_batches_tracked")]
    assert len(nbt) == n_bn and all(sh[k] == () for k in nbt)
    # state_dict order: a BN's buffers follow its bias
    ks = list(sh)
    i = ks.index("bn1.bias")
    assert ks[i + 1:i + 4] == ["bn1.running_mean", "bn1.running_var", "bn1.num_batches_tracked"]


def test_per_key_ciphertext_count_resnet18_batch4096():
    """The reference run (benchmark.py:423 model = model_res18, CKKS batch 4096 :477) encrypts every
    state_dict key on its own (:489-493): sum_k ceil(n_k / 4096) ciphertexts per client.  The 62
    parameter keys give 2,893; the 60 BN buffer keys (each <= 512 values) one ciphertext each."""
    params_only = sum(-(-int(np.prod(s)) // 4096) for s in F.resnet_shapes(18, buffers=False).values())
    assert params_only == 2893
    per_key = F.cts_per_key(F.resnet_shapes(18), 4096)
    assert sum(per_key.values()) == 2953 == params_only + 60
    assert per_key["layer4.1.bn2.num_batches_tracked"] == 1 and per_key["fc.weight"] == 125
    st = F.synthetic_states(F.resnet_shapes(18), 1, seed=1)[0]
    assert st["bn1.num_batches_tracked"].dtype == np.int64 and st["bn1.num_batches_tracked"].shape == (1,)
    assert (st["layer1.0.bn1.running_var"] >= 0).all()


def test_layer_index_rule():
    # benchmark_selection.py:152: re.sub("[^0-9]", "", key)
    assert F.layer_index("layer1.0.conv1.weight") == 101
    assert F.layer_index("fc.weight") is None
    assert F.layer_index("conv2.bias") == 2


def test_selection_modes():
    s = F.Selection("layers", layers=[2])
    assert s.encrypted_index("conv2.weight", 10) == slice(0, 10)
    assert s.encrypted_index("conv1.weight", 10) is None
    r = F.Selection("rate", rate=0.1)
    assert r.encrypted_index("x", 1000) == slice(0, 100)  # round(len * sel_rate)
    assert r.encrypted_index("x", 4) is None
    m = F.Selection("mask", masks={"a": np.array([True, False, True])})
    assert m.encrypted_index("a", 3).tolist() == [True, False, True]
    assert m.encrypted_index("b", 3) is None


def test_top_k_mask():
    sens = np.array([0.1, 5.0, 0.3, 4.0, 0.2])
    assert F.top_k_mask(sens, 0.4).tolist() == [False, True, False, True, False]


def _topk_indices(v, k):
    """torch.topk(v, k, largest=True).indices as a set, restated for tie-free v: the indices of
    the k largest values (a full descending sort, the first k)."""
    order = sorted(range(len(v)), key=lambda i: -float(v[i]))
    return set(order[:k])


@pytest.mark.parametrize("n,p", [(5, 0.5), (7, 0.3), (10, 0.25), (9, 0.95), (1000, 0.4), (3, 0.1),
                                 (161, 0.1), (11, 1.0), (4, 0.0)])
def test_top_k_mask_count_and_index_set(n, p):
    """masking.py:17: k = int(len(vector) * p), the floor -- 5 * 0.5 = 2.5 -> 2, 7 * 0.3 -> 2,
    9 * 0.95 = 8.55 -> 8 (round() would take one more) -- and the encrypted set is exactly
    topk's index set on tie-free input."""
    v = np.random.default_rng(n).permutation(n).astype(np.float64) * 0.37 + 0.01
    mask = F.top_k_mask(v, p)
    k = int(len(v) * p)
    assert int(mask.sum()) == k
    assert set(np.flatnonzero(mask).tolist()) == _topk_indices(v, k)
    torch = pytest.importorskip("torch")
    t = torch.from_numpy(v)
    assert set(np.flatnonzero(mask).tolist()) == set(torch.topk(t, k, largest=True).indices.tolist())


def test_flatten_roundtrip():
    torch = pytest.importorskip("torch")
    st = {"w": torch.randn(3, 4), "b": torch.randn(4)}
    flat = F.flatten_state(st)
    assert flat["w"].dtype == np.float64 and flat["w"].shape == (12,)
    back = F.unflatten_state(flat, F.state_shapes(st), like=st)
    assert torch.equal(back["w"], st["w"]) and back["w"].dtype == torch.float32


def test_plain_fedavg():
    sts = F.synthetic_states(F.lenet5_shapes(), 3, seed=1)
    w = [0.2, 0.3, 0.5]
    got = F.plain_fedavg(sts, w, "fc1.weight")
    assert np.allclose(got, sum(wi * s["fc1.weight"] for wi, s in zip(w, sts)))
