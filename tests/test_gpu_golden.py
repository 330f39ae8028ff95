"""The HIP path against the committed golden vectors: the same seeded FedAvg round
through SHELFI_FHE (keygen / loadCryptoParams, encrypt, computeWeightedAverage,
decrypt) reproduces the oracle's fixture bit for bit."""
import os

import numpy as np
import pytest

import golden_cases as G
from conftest import PALISADE_DIR
from test_golden import check_round, load

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402


@pytest.mark.parametrize("name", sorted(G.CASES))
def test_product_reproduces_golden(name, tmp_path):
    rec, arrays = load(name)
    slots, depth, kseed, n = G.CASES[name]
    if kseed is None:
        ck = m.CKKS("ckks", slots, 52, PALISADE_DIR, decodeNoise=False)
        ck.loadCryptoParams()
    else:
        ck = m.CKKS("ckks", slots, 52, str(tmp_path) + os.sep, multDepth=depth, seed=kseed, decodeNoise=False)
        assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    N, L = inf["ring_dim"], inf["num_towers"]
    assert inf["moduli"] == rec["moduli"]
    ck.set_seed(G.ENC_SEED)
    blobs = [ck.encrypt(x) for x in G.learner_inputs(n)]  # learner i -> counters i*K..
    agg_blob = ck.computeWeightedAverage(blobs, G.weights())
    dec = ck.decrypt(agg_blob, n)
    pk, sk = ck.get_keys()
    cts = [m.blob_residues(b, N, L) for b in blobs]
    check_round(rec, arrays, pk, sk, cts, m.blob_residues(agg_blob, N, L), dec)
