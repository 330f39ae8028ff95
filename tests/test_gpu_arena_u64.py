"""The arena's uint64 layout (round 4): Arena(..., layout="auto") keeps small
arenas (<= Arena.AUTO_U64_ROWS rows of 512 residues per learner, cfg2's 2,048) as C uint64
learner batches aggregated by wavg_kernel, whose 4x shorter waves fill the chip where one packed
wave per row cannot.  Same contract as the packed layout: every put is validated (uploads'
headers against the context, every residue < q_t), a refused slot blocks wavg until rewritten,
and the aggregate is bit-identical to the packed arena's and the oracle's."""
import os

import numpy as np
import pytest

import oracle as O
from conftest import PALISADE_DIR, PALISADE_PYBIND_DIR

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402
from SHELFI_FHE import dist as X  # noqa: E402


@pytest.fixture(scope="module")
def c2(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("u64_c2")) + os.sep
    ck = m.CKKS("ckks", 16384, 52, d, multDepth=3, seed=7, decodeNoise=False, wireFormat="shelfi")
    assert ck.genCryptoContextAndKeyGen() == 1
    return ck


def test_auto_layout_by_rows(c2):
    """cfg2's 16 x 4 arena (2,048 rows per learner) takes the uint64 layout; cfg5-sized ones stay packed."""
    assert D.Arena(c2, 16, 4, layout="auto").layout == "uint64"
    assert D.Arena(c2, 16, 4).layout == "packed"  # the default; "auto" is opt-in
    assert D.Arena(c2, 2, 8, layout="auto").layout == "uint64"   # 4,096 rows: the threshold itself
    assert D.Arena(c2, 2, 9, layout="auto").layout == "packed"
    assert D.Arena(c2, 2, 1, layout="packed").layout == "packed"
    with pytest.raises(ValueError):
        D.Arena(c2, 2, 1, layout="u128")


@pytest.mark.parametrize("C,K", [(16, 4), (3, 2), (20, 1)])
def test_u64_layout_matches_packed_and_oracle(c2, C, K):
    inf = c2.info()
    B, q, delta = inf["batch"], np.array(inf["moduli"], np.uint64), inf["delta"]
    rng = np.random.default_rng(C * 10 + K)
    xs = [rng.uniform(-1, 1, K * B - 9) for _ in range(C)]
    cts = [D.encrypt(c2, torch.from_numpy(x).cuda()) for x in xs]
    blob = c2.encrypt(xs[1])
    w = list(rng.dirichlet(np.ones(C)))
    au = D.Arena(c2, C, K, layout="uint64")
    ap = D.Arena(c2, C, K, layout="packed")
    res = [c.cpu().numpy().view(np.uint64) for c in cts]
    res[1] = m.blob_residues(blob, inf["ring_dim"], inf["num_towers"])  # learner 1 arrives as an upload
    for i, c in enumerate(cts):
        au.put(i, c if i != 1 else blob)
        ap.put(i, c if i != 1 else blob)
    ref = O.wavg(res, w, q, delta)
    got = au.wavg(w)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint64), ref)
    assert torch.equal(got, ap.wavg(w))
    if K > 1:
        assert torch.equal(au.wavg(w, k0=1, k1=K), ap.wavg(w, k0=1, k1=K))
    out, ms = au.place_output(w)
    assert ms == [] and torch.equal(out, got)
    with pytest.raises(ValueError, match="packed"):
        au.wavg_packed(w)


def test_u64_layout_refusals(c2, tmp_path):
    inf = c2.info()
    B = inf["batch"]
    K = 2
    xs = [np.random.default_rng(i).uniform(-1, 1, K * B) for i in range(2)]
    cts = [D.encrypt(c2, torch.from_numpy(x).cuda()) for x in xs]
    ar = D.Arena(c2, 2, K, layout="uint64")
    ar.put(0, cts[0])
    ar.put(1, cts[1])
    good = ar.wavg([0.5, 0.5]).clone()
    bad = cts[0].clone()
    bad[1, 1, 2, 7] = int(inf["moduli"][2])  # == q_t: not canonical
    with pytest.raises(m.ShelfiError, match="residue"):
        ar.put(0, bad)
    with pytest.raises(m.ShelfiError, match="refused upload for learner 0"):
        ar.wavg([0.5, 0.5])
    ar.put(0, cts[0])
    assert torch.equal(ar.wavg([0.5, 0.5]), good)
    # an upload under another key is refused at its header and marks the slot too
    other = m.CKKS("ckks", 16384, 52, str(tmp_path) + os.sep, multDepth=3, seed=8, decodeNoise=False,
                   wireFormat="shelfi")
    assert other.genCryptoContextAndKeyGen() == 1
    with pytest.raises(m.ShelfiError, match="different key"):
        ar.put(1, other.encrypt(xs[1]))
    with pytest.raises(m.ShelfiError, match="refused upload for learner 1"):
        ar.wavg([0.5, 0.5])
    ar.put(1, cts[1])
    assert torch.equal(ar.wavg([0.5, 0.5]), good)
    # slot() is a copy: writing into it cannot place an unvalidated residue in the arena
    s0 = ar.slot(0)
    assert torch.equal(s0, cts[0])
    s0.fill_(-1)
    assert torch.equal(ar.slot(0), cts[0]) and torch.equal(ar.wavg([0.5, 0.5]), good)
    # the C-ABI combine takes packed arenas only
    comm = X.Comm(c2, rank=0, world=1)
    try:
        with pytest.raises(ValueError, match="packed"):
            comm.combine_arena(ar, [0.5, 0.5], K, D.empty_ct(c2, K), D.empty_ct(c2, K))
    finally:
        comm.close()


def test_check_residues_entry_point(c2):
    inf = c2.info()
    ct = D.encrypt(c2, torch.rand(3 * inf["batch"], device="cuda", dtype=torch.float64))
    lib = m._lib.load()
    import ctypes as C

    assert lib.shelfi_dev_check_residues(c2._ctx, C.c_void_p(ct.data_ptr()), 3, None) == 0
    ct[2, 1, 3, -1] = -1  # 2^64 - 1
    assert lib.shelfi_dev_check_residues(c2._ctx, C.c_void_p(ct.data_ptr()), 3, None) == m._lib.SHELFI_ERR_FORMAT
