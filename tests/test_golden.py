"""The oracle against the committed golden vectors (tests/golden/vectors, written by
tests/golden/make_vectors.py): one seeded FedAvg round per parameter set — keys,
every learner's ciphertexts, the aggregate and the decode — must reproduce bit for
bit, and the decode must be within CKKS error of plain FedAvg."""
import json
import os

import numpy as np
import pytest

import golden_cases as G
import oracle as O
from conftest import ROOT

VEC = os.path.join(ROOT, "tests", "golden", "vectors")


def load(name):
    with open(os.path.join(VEC, name + ".json")) as f:
        rec = json.load(f)
    arrays = None
    p = os.path.join(VEC, name + ".npz")
    if os.path.exists(p):
        with np.load(p, allow_pickle=False) as z:
            arrays = {k: z[k] for k in z.files}
    return rec, arrays


def check_round(rec, arrays, pk, sk, cts, agg, dec):
    assert G.sha256(pk) == rec["pk_sha256"] and G.sha256(sk) == rec["sk_sha256"]
    assert [G.sha256(c) for c in cts] == rec["ct_sha256"]
    assert list(agg.shape) == rec["agg_shape"]
    for i, v in rec["agg_samples"]:
        assert int(agg[tuple(i)]) == v
    for i, v in rec["ct0_samples"]:
        assert int(cts[0][tuple(i)]) == v
    for j, v in rec["dec_samples"]:
        assert float(dec[j]) == v
    assert G.sha256(agg) == rec["agg_sha256"]
    assert G.sha256(dec) == rec["dec_sha256"]
    if arrays is not None:
        assert np.array_equal(cts[0], arrays["ct0"])
        assert np.array_equal(agg, arrays["agg"])
        assert np.array_equal(dec, arrays["dec"])


@pytest.mark.parametrize("name", sorted(G.CASES))
def test_oracle_reproduces_golden(name, palisade_keys):
    rec, arrays = load(name)
    pk, sk, cts, agg, dec, q, psi = G.oracle_round(O, name, palisade_keys)
    assert [int(x) for x in q] == rec["moduli"]
    check_round(rec, arrays, pk, sk, cts, agg, dec)
    # CKKS error at Delta ~ 2^52 after one EvalMult: far below 1e-7
    n = G.CASES[name][3]
    assert np.abs(dec - G.plain_fedavg(n)).max() < 1e-8
    assert rec["max_abs_err_vs_plain_fedavg"] < 1e-8


def test_cfg1_fixture_is_under_the_reference_keys(palisade_keys):
    """cfg1's ciphertexts decrypt under the reference's committed private key."""
    rec, arrays = load("cfg1")
    ctx, pk, sk = palisade_keys
    q = np.array(ctx["q"], np.uint64)
    psi = np.array(ctx["psi"], np.uint64)
    x0 = G.learner_inputs(1000)[0]
    d = O.decrypt(arrays["ct0"][0], sk, q, psi, 4096, float(int(q[-1])), 1000)
    assert np.abs(d - x0).max() < 1e-8
