"""§8(f3): PALISADE 1.11 decode noise flooding, restated in the oracle
(or_decode_stats / or_decode_symmetrize / or_decrypt_flood).  The estimator and the
thresholds are checked on synthetic coefficient pairs with a known error; the
flooded decrypt of a real ciphertext under the reference keys stays within the
added noise of the exact decode.  Normalisation constants of PALISADE's StdDev are
restated, not pinned (PALISADE absent): parity with PALISADE is tolerance-level."""
import numpy as np
import pytest

import oracle as O

P_BITS = 52


def _pairs(S, N, sigma_p, rng, sym_scale=0.5):
    """Coefficient pairs = a symmetric message part + an error with per-coefficient
    stddev sigma_p (at scale 2^p), expressed in output units."""
    # symmetric part: m(X) = m(X^-1) <=> re_i = -im_{S-i}, im_0 = 0, re_h = -im_h
    re = rng.uniform(-sym_scale, sym_scale, S)
    im = np.empty(S)
    im[0] = 0.0
    im[1:] = -re[1:][::-1]
    h = S // 2
    im[h] = -re[h]
    e = rng.normal(0, sigma_p, (2, S)) / 2.0 ** P_BITS
    return re + e[0], im + e[1]


@pytest.mark.parametrize("S,N", [(4096, 8192), (16384, 32768), (1024, 8192)])
def test_sigma_estimate_recovers_known_error(S, N):
    rng = np.random.default_rng(S)
    for sigma_p in (40.0, 3000.0, 2.0 ** 30):
        re, im = _pairs(S, N, sigma_p, rng)
        sd, le, fail = O.decode_stats(re, im, N, P_BITS, 1.0)
        # u = v - conj has stddev sqrt(2) sigma_p; 0.5 sqrt(var) = sigma_p / sqrt(2)
        est = sd / np.sqrt(2.0)
        assert abs(est - sigma_p / np.sqrt(2.0)) / (sigma_p / np.sqrt(2.0)) < 0.05, (sigma_p, est)
        assert not fail
        assert le == int(np.rint(np.log2(sd * np.sqrt(2 * S))))


def test_sigma_floor_and_precision_failure():
    rng = np.random.default_rng(1)
    S, N = 4096, 8192
    re, im = _pairs(S, N, 0.0, rng)  # exact symmetric message: floor sqrt(N)/8
    sd, le, fail = O.decode_stats(re, im, N, P_BITS, 1.0)
    assert sd == pytest.approx(np.sqrt(2.0) * 0.125 * np.sqrt(N)) and not fail
    re, im = _pairs(S, N, 2.0 ** 48, rng)  # ~4 bits of precision left -> PALISADE throws
    assert O.decode_stats(re, im, N, P_BITS, 1.0)[2]
    sd3, _, _ = O.decode_stats(*_pairs(S, N, 1000.0, rng), N, P_BITS, 3.0)
    sd1, _, _ = O.decode_stats(*_pairs(S, N, 1000.0, np.random.default_rng(1)), N, P_BITS, 1.0)
    assert sd3 / sd1 == pytest.approx(np.sqrt(4.0 / 2.0), rel=0.1)  # sqrt(M + 1)


def test_flooded_decrypt_of_a_real_ciphertext(palisade_keys):
    ctx, pk, sk = palisade_keys
    q = np.array(ctx["q"], np.uint64)
    psi = np.array(ctx["psi"], np.uint64)
    N, S = ctx["N"], 4096
    delta = float(int(q[-1]))
    x = np.random.default_rng(2).uniform(-1, 1, S).astype(np.float32).astype(np.float64)
    ct = O.encrypt_vector(x, pk, q, psi, N, S, delta, seed=11)[0]
    exact = O.decrypt(ct, sk, q, psi, S, delta, S)
    fl, le, fail = O.decrypt_flood(ct, sk, q, psi, S, delta, S, seed=11, g=5)
    assert not fail
    re, im = O.decrypt_coeffs(ct, sk, q, psi, S, delta)
    sd, le2, _ = O.decode_stats(re, im, N, P_BITS, 1.0)
    assert le == le2
    # slot noise: real part of an S-term sum of iid N(0, nsd^2) pairs -> nsd sqrt(S)
    nsd = sd / 2.0 ** P_BITS
    d = fl - exact
    assert np.std(d) == pytest.approx(nsd * np.sqrt(S), rel=0.1)
    assert np.abs(d).max() < 8 * nsd * np.sqrt(S)
    assert np.abs(fl - x).max() < 1e-9
    # the seeded stream is reproducible, another ciphertext index draws other noise
    assert np.array_equal(O.decrypt_flood(ct, sk, q, psi, S, delta, S, seed=11, g=5)[0], fl)
    assert not np.array_equal(O.decrypt_flood(ct, sk, q, psi, S, delta, S, seed=11, g=6)[0], fl)


def test_fft_special_is_sqrt_s_times_unitary():
    """Round 5 moved the decode noise to the output domain (or_flood_out_normals).  That is
    distribution-preserving because FFTSpecial's matrix F satisfies F F^H = S I: PALISADE's i.i.d.
    circular complex input noise z (unit variance per component) maps to F z, whose real parts have
    covariance (Re(F E[z z^H] F^H) + Re(F E[z z^T] F^T)) / 2 = S I: i.i.d. N(0, S)."""
    for S in (64, 256):
        F = np.stack([O.fft_special(np.eye(S)[j] + 0j) for j in range(S)], axis=1)  # column j = F e_j
        assert np.abs(F @ F.conj().T - S * np.eye(S)).max() < 1e-9 * S
        # z circular (E z z^T = 0): Cov(Re F z) = Re(F F^H) / 2 per unit component variance x 2 = S I


def test_output_domain_noise_matches_input_domain_distribution():
    """The input-domain form (PALISADE's order: symmetrize, add N(0, nsd) to every FFT input, decode)
    and the output-domain form (exact decode + N(0, nsd sqrt(S)) per slot) have the same
    per-slot standard deviation and no cross-slot correlation (Monte Carlo at S = 256)."""
    S, nsd, trials = 256, 1.0, 400
    rng = np.random.default_rng(7)
    samples = []
    for _ in range(trials):
        z = rng.standard_normal(S) + 1j * rng.standard_normal(S)
        samples.append(O.fft_special(nsd * z).real)
    a = np.array(samples)
    assert np.std(a) == pytest.approx(nsd * np.sqrt(S), rel=0.05)
    c = np.corrcoef(a[:, :8].T)
    assert np.abs(c - np.eye(8)).max() < 0.2


def test_output_domain_normals_stream():
    """or_flood_out_normals: slot i takes normal (i div S/16) of block (i mod S/16); standard normal."""
    S = 4096
    z = O.flood_out_normals(11, 5, S)
    assert z.shape == (S,) and abs(np.mean(z)) < 0.1 and np.std(z) == pytest.approx(1.0, rel=0.05)
    key = O.seed_to_key(11)
    blk = O.chacha20_block(key, 7, (3 << 56) | 5)
    u1 = (float(blk[2]) + 1.0) * 2.0 ** -32
    u2 = float(blk[3]) * 2.0 ** -32
    r = np.sqrt(-2 * np.log(u1))
    assert z[7 + (S // 16) * 2] == pytest.approx(r * np.cos(2 * np.pi * u2), abs=1e-15)
    assert z[7 + (S // 16) * 3] == pytest.approx(r * np.sin(2 * np.pi * u2), abs=1e-15)
