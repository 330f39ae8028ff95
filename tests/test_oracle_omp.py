"""The CPU baseline's all-core encrypt / decrypt: the oracle's OpenMP loops over
ciphertexts (the reference's `#pragma omp parallel for`, ckks.cpp:70 and :186) give the same
ciphertexts and values as the one-ciphertext-at-a-time restatement, at any thread count."""
import numpy as np
import pytest

import oracle as O


@pytest.mark.parametrize("threads", [1, 3])
def test_omp_encrypt_decrypt_equal_the_serial_oracle(threads):
    N, L, S = 1 << 13, 2, 4096
    q, psi = O.params_generate(N, L)
    rng = np.random.default_rng(threads)
    pk = np.stack([np.stack([rng.integers(0, int(q[t]), N, dtype=np.uint64) for t in range(L)])
                   for _ in range(2)])
    x = rng.uniform(-1, 1, 3 * S + 5)
    delta = float(q[-1])
    a = O.encrypt_vector(x, pk, q, psi, N, S, delta, seed=5, g0=3)
    b = O.encrypt_vector_omp(x, pk, q, psi, N, S, delta, seed=5, g0=3, nthreads=threads)
    assert np.array_equal(a, b)
    s = rng.integers(-1, 2, N)
    sk = np.stack([O.ntt_fwd((s % int(q[t])).astype(np.uint64), q[t], psi[t]) for t in range(L)])
    for n in (len(x), 2 * S - 1):
        d1 = O.decrypt_vector(a, sk, q, psi, S, delta, n)
        d2 = O.decrypt_vector_omp(a, sk, q, psi, S, delta, n, nthreads=threads)
        assert np.array_equal(d1, d2)
