"""GPU: the encrypted FedAvg harness (SHELFI_FHE.fedavg) against plain FedAvg, for
every selection mode of the reference's harnesses (benchmark.py, benchmark_selection.py,
benchmark_selection_rate.py, masking.py).  Tolerance 1e-7 absolute (CKKS at Delta~2^52)."""
import numpy as np
import pytest

from conftest import PALISADE_DIR

pytestmark = pytest.mark.gpu

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import fedavg as F  # noqa: E402


@pytest.fixture(scope="module")
def ck():
    c = m.CKKS("ckks", 4096, 52, PALISADE_DIR, seed=5, decodeNoise=False)
    c.loadCryptoParams()
    return c


@pytest.mark.parametrize("mode,pack", [("all", False), ("all", True), ("layers", False), ("rate", False),
                                       ("mask", False), ("mask", True)])
def test_secure_fedavg_lenet(ck, mode, pack):
    states = F.synthetic_states(F.lenet5_shapes(), 3, seed=3)
    w = [0.5, 0.2, 0.3]
    if mode == "layers":
        sel = F.Selection("layers", layers=[1, 3])
    elif mode == "rate":
        sel = F.Selection("rate", rate=0.1)
    elif mode == "mask":
        rng = np.random.default_rng(0)
        sel = F.Selection("mask", masks={k: F.top_k_mask(rng.random(v.size), 0.1) for k, v in states[0].items()})
    else:
        sel = F.Selection("all")
    agg, times = F.SecureFedAvg(ck, sel, pack=pack).run(states, w)
    for k in states[0]:
        exp = sum(float(np.float32(wi)) * s[k] for wi, s in zip(w, states))
        assert np.abs(agg[k] - exp).max() < 1e-7, k
    assert times["aggregate"] > 0


def test_secure_fedavg_resnet18_state_dict_per_key(ck):
    """benchmark.py:447-543 as the reference runs it: ResNet-18's whole state_dict (122 keys with
    the BN buffers, int64 num_batches_tracked included, widened by encrypt's forcecast) encrypted
    key by key at batch 4096 — exactly 2,953 ciphertexts per client — aggregated and decrypted to
    each key's size."""
    states = F.synthetic_states(F.resnet_shapes(18), 3, seed=6)
    assert states[0]["bn1.num_batches_tracked"].dtype == np.int64
    sf = F.SecureFedAvg(ck)
    counts = {}
    real_encrypt = ck.encrypt

    def counting_encrypt(x):
        b = real_encrypt(x)
        counts[len(counts)] = m.blob_info(b)["num_cts"]
        return b

    ck.encrypt = counting_encrypt
    try:
        agg, _ = sf.run(states)
    finally:
        del ck.encrypt
    assert len(counts) == 3 * 122 and sum(counts.values()) == 3 * 2953
    w32 = float(np.float32(1 / 3))
    for k in states[0]:
        exp = sum(s[k].astype(np.float64) for s in states) * w32
        assert agg[k].shape == exp.shape
        assert np.abs(agg[k] - exp).max() < 1e-7 * max(1.0, float(np.abs(exp).max())), k


def test_secure_fedavg_resnet18_packed(ck):
    """ResNet-18's state_dict (11,699,132 values, 2,857 ciphertexts at batch 4096), 3 clients."""
    states = F.synthetic_states(F.resnet_shapes(18), 3, seed=4)
    agg, _ = F.SecureFedAvg(ck, pack=True).run(states)
    for k in ("conv1.weight", "layer4.1.conv2.weight", "fc.bias"):
        exp = sum(s[k] for s in states) * float(np.float32(1 / 3))
        assert np.abs(agg[k] - exp).max() < 1e-7, k
